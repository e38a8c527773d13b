cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 0 3; do timeout -k 10 300 python -u scripts/ab_grid.py $v > gpurun_out/ab_grid_$v.log 2>&1 || { echo "ab rc=$?"; tail gpurun_out/ab_grid_$v.log; exit 1; }; grep var gpurun_out/ab_grid_$v.log; done
