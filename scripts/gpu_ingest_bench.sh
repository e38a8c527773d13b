cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --config 2 --keys 1000000 --ingest --cpu-keys 0 --steps 2 --warmup 1 > gpurun_out/bench_ingest.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/bench_ingest.log; exit 1; }
tail -1 gpurun_out/bench_ingest.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ingest'])"
