cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mirror.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gst or GST or rccl or select" > gpurun_out/pytest_gst.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/pytest_gst.log; exit 1; }
tail -1 gpurun_out/pytest_gst.log
timeout -k 10 300 python -u bench.py --config 2 --gst --cpu-keys 0 --steps 3 --warmup 1 > gpurun_out/bench_gst.log 2>&1 || { echo "bench rc=$?"; tail gpurun_out/bench_gst.log; exit 1; }
tail -1 gpurun_out/bench_gst.log | python3 -c "import sys,json; print(json.loads(sys.stdin.read())['gst'])"
