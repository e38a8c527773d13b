cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/ab_env.py --cfg 3 --cfg 4 --rounds 8 --var def: --var nt:AGN_TAGS_EXP=1 --var filt_x:AGN_TAGS_EXP=2 --var filtnt_x:AGN_TAGS_EXP=3 > gpurun_out/ab_tags_exp.log 2>&1 || { echo "ab rc=$?"; tail gpurun_out/ab_tags_exp.log; exit 1; }
grep -E "cfg" gpurun_out/ab_tags_exp.log
