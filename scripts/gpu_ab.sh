# A/B of the counter kernel variants in one process + default bench line.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/ab_counter.py > gpurun_out/ab_counter.log 2>&1 || { echo "ab rc=$?"; tail gpurun_out/ab_counter.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_counter.log
timeout -k 10 400 python -u bench.py --cpu-keys 0 > gpurun_out/bench_default.log 2>&1 || { echo "bench rc=$?"; tail gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
