cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
timeout -k 10 300 python -u scripts/ab_env.py --cfg 2 --rounds 8 --var w2:AGN_COUNTER_WPB=2 --var w1:AGN_COUNTER_WPB=1 --var w4:AGN_COUNTER_WPB=4 > gpurun_out/ab_wpb_$r.log 2>&1 || { echo "rc=$?"; tail -30 gpurun_out/ab_wpb_$r.log; exit 1; }
grep cfg gpurun_out/ab_wpb_$r.log
done
