cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "auto-2- or auto-3- or long or large or repeated or cfg3 or cfg4 or system" > gpurun_out/pytest_tags.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/pytest_tags.log; exit 1; }
tail -1 gpurun_out/pytest_tags.log
for r in 1 2; do
for L in tools/ab/lib_prev.so antidote_amd/libantidote_gpu.so; do
AGN_LIB=$L timeout -k 10 300 python -u scripts/ab_tags.py > gpurun_out/ab_tags_x.log 2>&1 || { echo "ab rc=$?"; tail gpurun_out/ab_tags_x.log; exit 1; }
echo "$L"; grep cfg gpurun_out/ab_tags_x.log
done; done
