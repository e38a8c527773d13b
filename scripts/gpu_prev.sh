# Current library vs tools/libagn_prev.so (scripts/build_prev.sh), cfg2 twice + cfg3/cfg4, after the counter parity tests.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_id_index.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "index or id0 or random or full_size or generator or long or kat" > gpurun_out/pytest_prev.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/pytest_prev.log; exit 1; }
tail -1 gpurun_out/pytest_prev.log
for c in 2 2 ${AB_EXTRA:-}; do
timeout -k 10 300 python -u scripts/ab_prev.py $c > gpurun_out/ab_prev_$c.log 2>&1 || { echo "ab rc=$?"; tail gpurun_out/ab_prev_$c.log; exit 1; }
grep cfg gpurun_out/ab_prev_$c.log
done
