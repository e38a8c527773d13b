# Tag-resolution kernel: parity + cfg3/cfg4 bench.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not counter_pn and (random or long or large or repeated or cfg3 or cfg4 or kat)" > gpurun_out/pytest_tags.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/pytest_tags.log; exit 1; }
tail -3 gpurun_out/pytest_tags.log
timeout -k 10 300 python -u bench.py --config 3 --steps 5 --warmup 1 --cpu-keys 0 > gpurun_out/bench3.log 2>&1 || { echo "bench3 rc=$?"; tail gpurun_out/bench3.log; exit 1; }
tail -1 gpurun_out/bench3.log
timeout -k 10 300 python -u bench.py --config 4 --steps 5 --warmup 1 --cpu-keys 0 > gpurun_out/bench4.log 2>&1 || { echo "bench4 rc=$?"; tail gpurun_out/bench4.log; exit 1; }
tail -1 gpurun_out/bench4.log
