cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/ab_xcd.py 2 3 4 > gpurun_out/ab_xcd.log 2>&1 || { echo "rc=$?"; tail -30 gpurun_out/ab_xcd.log; exit 1; }
grep cfg gpurun_out/ab_xcd.log
