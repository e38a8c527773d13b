cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/ab_b2b.py > gpurun_out/ab_b2b.log 2>&1 || { echo "rc=$?"; tail -30 gpurun_out/ab_b2b.log; exit 1; }
grep -E "round|probe" gpurun_out/ab_b2b.log
timeout -k 10 300 python -u scripts/ab_env.py --cfg 2 --var vgpr:AGN_COUNTER_GLDS=0 --var glds:AGN_COUNTER_GLDS=1 > gpurun_out/ab_glds2.log 2>&1 || { echo "rc=$?"; tail -30 gpurun_out/ab_glds2.log; exit 1; }
grep cfg gpurun_out/ab_glds2.log
timeout -k 10 300 python -u scripts/ab_env.py --cfg 2 --var glds:AGN_COUNTER_GLDS=1 --var vgpr:AGN_COUNTER_GLDS=0 > gpurun_out/ab_glds3.log 2>&1 || { echo "rc=$?"; tail -30 gpurun_out/ab_glds3.log; exit 1; }
grep cfg gpurun_out/ab_glds3.log
timeout -k 10 300 python -u bench.py --cpu-keys 0 > gpurun_out/bench_g1.log 2>&1 && tail -c 700 gpurun_out/bench_g1.log
AGN_COUNTER_GLDS=0 timeout -k 10 300 python -u bench.py --cpu-keys 0 > gpurun_out/bench_g0.log 2>&1 && tail -c 700 gpurun_out/bench_g0.log
