cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_tags.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/pytest_tags.log; exit 1; }
tail -1 gpurun_out/pytest_tags.log
: > gpurun_out/ab_tags3.log
for r in 1 2; do
for L in tools/ab/lib_prev.so antidote_amd/libantidote_gpu.so; do
echo "== $L" >> gpurun_out/ab_tags3.log
AGN_LIB=$L timeout -k 10 300 python -u scripts/ab_env.py --cfg 3 --cfg 4 --rounds 8 --var def: >> gpurun_out/ab_tags3.log 2>&1 || { echo "ab rc=$?"; tail gpurun_out/ab_tags3.log; exit 1; }
done; done
grep -E "==|cfg" gpurun_out/ab_tags3.log
