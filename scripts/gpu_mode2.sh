cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
( hostname; rocm-smi --showmemvendor --showvbios 2>&1 | grep -iE "vendor|vbios version" ) > gpurun_out/boxinfo.txt 2>&1 || true
cat gpurun_out/boxinfo.txt
for r in 1 2 3; do
timeout -k 10 300 python -u scripts/ab_env.py --cfg 2 --rounds 6 --var vgpr:AGN_COUNTER_GLDS=0 --var m0:AGN_COUNTER_MODE=0 --var m10:AGN_COUNTER_MODE=10 > gpurun_out/ab_mode2_$r.log 2>&1 || { echo "rc=$?"; tail -30 gpurun_out/ab_mode2_$r.log; exit 1; }
grep cfg gpurun_out/ab_mode2_$r.log
done
