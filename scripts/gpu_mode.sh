cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
( hostname; rocm-smi --showproductname --showmemvendor --showclocks --showfwinfo --showvbios --showdriverversion 2>&1; rocminfo 2>&1 | grep -iE "marketing|uuid|max clock|compute unit" | head -20 ) > gpurun_out/boxinfo.txt 2>&1 || true
timeout -k 10 400 python -u scripts/ab_env.py --cfg 2 --rounds 10 --var vgpr:AGN_COUNTER_GLDS=0 --var m0:AGN_COUNTER_MODE=0 --var m1:AGN_COUNTER_MODE=1 --var m4:AGN_COUNTER_MODE=4 --var m5:AGN_COUNTER_MODE=5 --var m2:AGN_COUNTER_MODE=2 --var m8:AGN_COUNTER_MODE=8 --var m10:AGN_COUNTER_MODE=10 > gpurun_out/ab_mode.log 2>&1 || { echo "rc=$?"; tail -30 gpurun_out/ab_mode.log; exit 1; }
grep cfg gpurun_out/ab_mode.log
grep -iE "vendor|mclk|fclk|sclk|VBIOS|driver|Marketing" gpurun_out/boxinfo.txt | head -20
