cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
( hostname; rocm-smi --showmemvendor --showvbios 2>&1 | grep -iE "vendor|vbios version" ) > gpurun_out/boxinfo.txt 2>&1 || true
cat gpurun_out/boxinfo.txt
timeout -k 10 300 python -u scripts/ab_env.py --cfg 2 --rounds 10 --var vgpr: --var ids:AGN_COUNTER_IDS=1 --var ids_w1:AGN_COUNTER_IDS=1,AGN_COUNTER_WPB=1 --var ids_w4:AGN_COUNTER_IDS=1,AGN_COUNTER_WPB=4 --var w1:AGN_COUNTER_WPB=1 --var glds:AGN_COUNTER_GLDS=1 > gpurun_out/ab_ids.log 2>&1 || { echo "rc=$?"; tail -30 gpurun_out/ab_ids.log; exit 1; }
grep cfg gpurun_out/ab_ids.log
