cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_counter.sh && bash scripts/gpu_ab.sh
