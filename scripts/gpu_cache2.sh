cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ss_cache.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_cache.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/pytest_cache.log; exit 1; }
tail -1 gpurun_out/pytest_cache.log
bash scripts/gpu_warm.sh
