# Counter dense kernel: parity + A/B of prefetch depth + default bench.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "auto-1- or general-1- or kat or cfg2 or long or empty" > gpurun_out/pytest_counter.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/pytest_counter.log; exit 1; }
tail -2 gpurun_out/pytest_counter.log
for v in 1 2 8; do AGN_COUNTER_WPB=$v timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "random and auto-1-" > gpurun_out/pytest_counter_v$v.log 2>&1 || { echo "pytest v$v rc=$?"; tail -40 gpurun_out/pytest_counter_v$v.log; exit 1; }; tail -1 gpurun_out/pytest_counter_v$v.log; done
timeout -k 10 300 python -u scripts/ab_counter.py > gpurun_out/ab_counter.log 2>&1 || { echo "ab rc=$?"; tail gpurun_out/ab_counter.log; exit 1; }
cat gpurun_out/ab_counter.log | grep -v amdgpu.ids
