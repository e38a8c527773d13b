# Optimisation round: parity with the dense kernel, A/B, bench, rocprof kernel
# trace + HBM PMC passes.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
: > gpurun_out/steps.txt
step pytest_gpu 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mirror.py -q --timeout 300 --timeout-method thread -m gpu
step ab 300 python -u scripts/ab_counter.py
step bench 600 python -u bench.py --steps 20 --warmup 3
step prof_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-keys 0
step prof_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-keys 0
step prof_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-keys 0
