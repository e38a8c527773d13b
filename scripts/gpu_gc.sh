cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_prune.py tests/test_next_rows.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gc.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/pytest_gc.log; exit 1; }
tail -1 gpurun_out/pytest_gc.log
timeout -k 10 300 python -u bench.py --config 2 --keys 1000000 --gc --cpu-keys 0 --steps 2 --warmup 1 > gpurun_out/bench_gc_small.log 2>&1 || { echo "bench small rc=$?"; tail -5 gpurun_out/bench_gc_small.log; exit 1; }
tail -1 gpurun_out/bench_gc_small.log | python3 -c "import sys,json; print(json.loads(sys.stdin.read())['gc'])"
for c in 2 3; do
timeout -k 10 300 python -u bench.py --config $c --gc --cpu-keys 0 --steps 3 --warmup 1 > gpurun_out/bench_gc$c.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/bench_gc$c.log; exit 1; }
tail -1 gpurun_out/bench_gc$c.log | python3 -c "import sys,json; print(json.loads(sys.stdin.read())['gc'])"
done
