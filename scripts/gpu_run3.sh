# Counter pipeline variants A/B + tags configs bench + parity.
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
step pytest_gpu 900 python -u -m pytest tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -m gpu -k "counter or random or long or KAT or kat"
step ab 300 python -u scripts/ab_counter.py
step bench3 600 python -u bench.py --config 3 --steps 5 --warmup 1 --cpu-keys 20000
step bench4 600 python -u bench.py --config 4 --steps 10 --warmup 2 --cpu-keys 20000
step prof_tags 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tags -o run -- python3 bench.py --config 3 --steps 3 --warmup 1 --cpu-keys 0
