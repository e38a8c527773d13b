# Baseline check: full GPU parity suite + default bench + smoke.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke rc=$?"; cat gpurun_out/smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench rc=$?"; tail gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
