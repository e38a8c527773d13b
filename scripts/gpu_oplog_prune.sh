# agn_oplog_prune: op-log GPU tests, then prev (CSR + re-segment) vs current
# (mark + direct segmented scatter) timing, alternating processes.
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
step oplog_tests 300 python -u -m pytest tests/test_oplog.py tests/test_batcher.py tests/test_prune.py -m gpu -x -q --timeout 120 --timeout-method thread
tail -2 gpurun_out/oplog_tests.log
for r in 1 2; do
  step prev$r 240 env AGN_LIB=tools/libagn_prev.so python -u scripts/bench_oplog_prune.py 500000 64 3
  step cur$r 240 python -u scripts/bench_oplog_prune.py 500000 64 3
done
cat gpurun_out/prev1.log gpurun_out/cur1.log gpurun_out/prev2.log gpurun_out/cur2.log | grep '^{'
