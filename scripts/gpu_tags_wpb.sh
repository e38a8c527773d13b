cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/ab_env.py --cfg 2 --rounds 12 --var w1:AGN_COUNTER_WPB=1 --var w2:AGN_COUNTER_WPB=2 --var w4:AGN_COUNTER_WPB=4 --var w1b:AGN_COUNTER_WPB=1 > gpurun_out/ab_wpb_def.log 2>&1 || { echo "rc=$?"; tail -30 gpurun_out/ab_wpb_def.log; exit 1; }
grep cfg gpurun_out/ab_wpb_def.log
timeout -k 10 400 python -u scripts/ab_env.py --cfg 3 --cfg 4 --rounds 8 --var w4:AGN_TAGS_WPB=4 --var w2:AGN_TAGS_WPB=2 --var w1:AGN_TAGS_WPB=1 --var w4b:AGN_TAGS_WPB=4 > gpurun_out/ab_tags_wpb.log 2>&1 || { echo "rc=$?"; tail -30 gpurun_out/ab_tags_wpb.log; exit 1; }
grep cfg gpurun_out/ab_tags_wpb.log
AGN_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --keys 1000000 --steps 5 --warmup 2 --cpu-keys 0 > gpurun_out/bench_n2_gloo.log 2>&1 || { echo "n2 rc=$?"; tail -30 gpurun_out/bench_n2_gloo.log; exit 1; }
grep metric gpurun_out/bench_n2_gloo.log | cut -c1-400
