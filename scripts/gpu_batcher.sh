cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_batcher.py tests/test_oplog.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_batcher.log 2>&1 || { echo "pytest rc=$?"; tail -60 gpurun_out/pytest_batcher.log; exit 1; }
tail -5 gpurun_out/pytest_batcher.log
