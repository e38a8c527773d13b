# key_id0 index: parity tests + A/B on cfg2 (twice, separate processes).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_id_index.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "index or id0 or random or full_size or generator or long or kat" > gpurun_out/pytest_id0.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/pytest_id0.log; exit 1; }
tail -2 gpurun_out/pytest_id0.log
timeout -k 10 300 python -u scripts/ab_id0.py > gpurun_out/ab_id0_a.log 2>&1 || { echo "ab rc=$?"; tail gpurun_out/ab_id0_a.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_id0_a.log
timeout -k 10 300 python -u scripts/ab_id0.py > gpurun_out/ab_id0_b.log 2>&1 || { echo "ab rc=$?"; tail gpurun_out/ab_id0_b.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_id0_b.log
