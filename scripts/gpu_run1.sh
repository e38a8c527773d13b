# GPU validation run: smoke, parity tests, full-size parity, bench.
# A test FAILURE (rc 1) continues; a timeout / crash / fault stops the call.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
: > gpurun_out/steps.txt
step smoke 240 python -u -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mirror.py -v --timeout 300 --timeout-method thread -k "not full_size" -m gpu
step pytest_full 700 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 400 --timeout-method thread -k "full_size" -m gpu
step bench 600 python -u bench.py --steps 10 --warmup 2
