cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "auto-1- or kat or cfg or long or empty or large or repeated or auto-2- or auto-3-" > gpurun_out/pytest_sel.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/pytest_sel.log; exit 1; }
tail -1 gpurun_out/pytest_sel.log
timeout -k 10 300 python -u scripts/ab_tags.py > gpurun_out/ab_tags.log 2>&1 || { echo "ab rc=$?"; tail gpurun_out/ab_tags.log; exit 1; }
grep cfg gpurun_out/ab_tags.log
