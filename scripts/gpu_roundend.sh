# Round-end rehearsal: the driver's GPU tiers (pytest -m gpu, smoke, default bench).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.txt
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -40 "gpurun_out/$name.log"; exit $rc; fi
  return 0
}
: > gpurun_out/steps.txt
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
tail -3 gpurun_out/pytest_gpu.log
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python -u bench.py
tail -n1 gpurun_out/bench.log
