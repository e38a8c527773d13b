# Tags kernel: 4 DCs per lane (default for dense D > 8) vs 8 (AGN_TAGS_DPL8=1), cfg3 + cfg4, after parity.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "dense_shapes or random or full_size or large or repeated or generator" > gpurun_out/pytest_dpl4.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/pytest_dpl4.log; exit 1; }
tail -1 gpurun_out/pytest_dpl4.log
for c in 3 4; do
timeout -k 10 300 python -u scripts/ab_prev.py $c dpl8=env:AGN_TAGS_DPL8=1 > gpurun_out/ab_dpl4_$c.log 2>&1 || { echo "ab rc=$?"; tail gpurun_out/ab_dpl4_$c.log; exit 1; }
grep cfg gpurun_out/ab_dpl4_$c.log
done
