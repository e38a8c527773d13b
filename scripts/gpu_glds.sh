cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_glds.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/pytest_glds.log; exit 1; }
tail -2 gpurun_out/pytest_glds.log
timeout -k 10 300 python -u scripts/ab_env.py --cfg 2 --var vgpr:AGN_COUNTER_GLDS=0 --var glds:AGN_COUNTER_GLDS=1 --var w1:AGN_COUNTER_WPB=1 --var w4:AGN_COUNTER_WPB=4 --var noxcd:AGN_XCD_REMAP=0 > gpurun_out/ab_glds.log 2>&1 || { echo "rc=$?"; tail -30 gpurun_out/ab_glds.log; exit 1; }
grep cfg gpurun_out/ab_glds.log
timeout -k 10 300 python -u scripts/ab_env.py --cfg 2 --warm 1 --var vgpr:AGN_COUNTER_GLDS=0 --var glds:AGN_COUNTER_GLDS=1 > gpurun_out/ab_glds_warm.log 2>&1 || { echo "rc=$?"; tail -30 gpurun_out/ab_glds_warm.log; exit 1; }
grep cfg gpurun_out/ab_glds_warm.log
