# Default-pool release threshold (AGN_POOL_KEEP): op-log / prune / ingest GPU
# tests, then agn_oplog_prune wall time with and without it, alternating.
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
step pool_tests 300 python -u -m pytest tests/test_oplog.py tests/test_batcher.py tests/test_prune.py tests/test_ingest.py -m gpu -x -q --timeout 120 --timeout-method thread
tail -2 gpurun_out/pool_tests.log
for r in 1 2; do
  step nokeep$r 240 env AGN_POOL_KEEP=0 python -u scripts/bench_oplog_prune.py 500000 64 5
  step keep$r 240 python -u scripts/bench_oplog_prune.py 500000 64 5
done
cat gpurun_out/nokeep1.log gpurun_out/keep1.log gpurun_out/nokeep2.log gpurun_out/keep2.log | grep '^{'
