cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/ab_probe.py > gpurun_out/ab_probe.log 2>&1 || { echo "rc=$?"; tail -30 gpurun_out/ab_probe.log; exit 1; }
cat gpurun_out/ab_probe.log
