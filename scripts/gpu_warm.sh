cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --config 2 --warm --cpu-keys 0 --steps 5 --warmup 1 > gpurun_out/bench_warm.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/bench_warm.log; exit 1; }
tail -1 gpurun_out/bench_warm.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['warm'], d['roofline']['kernel_ms'])"
