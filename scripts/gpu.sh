#!/bin/bash
# One parameterised GPU-box runner (replaces the per-experiment wrappers).
#
#   gpurun --timeout T -- bash scripts/gpu.sh 'name|seconds|command' ['name|seconds|command' ...]
#
# Each step runs from the repo root under its own `timeout -k 10 seconds`,
# with stdout+stderr in gpurun_out/<name>.log; the first failing step ends
# the script (no further GPU work after a fault, abort or time limit) and
# prints the tail of its log.  Recipes used every round:
#
#   roundend  : the driver's tiers -- pytest -m gpu, smoke(), default bench
#   trace     : rocprofv3 --kernel-trace --stats of the driver's exact bench
#               command (profiles/rNN/kernel_stats_*.csv)
#   pmc       : FETCH_SIZE / WRITE_SIZE passes (one counter block per run)
#   serve     : the native read/6 serving load generator (tools/serve_bench)
#
#   bash scripts/gpu.sh roundend        # expands to the three driver steps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/steps.txt

run_step() {
  local name=$1 t=$2 cmd=$3 soft=0
  # a name starting with '~': a plain failure (exit 1, e.g. a failed assert)
  # with no sign of a GPU error in its log does not end the script
  case "$name" in "~"*) soft=1; name=${name#"~"};; esac
  echo "[$(date +%T)] $name: $cmd" | tee -a gpurun_out/steps.txt
  timeout -k 10 "$t" bash -c "exec $cmd" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a gpurun_out/steps.txt
  if [ $rc -eq 1 ] && [ $soft -eq 1 ] && \
     ! grep -qiE "fault|hipError|HSA_STATUS|illegal|abort|core dumped|hip error|EHIP" "gpurun_out/$name.log"; then
    echo "$name failed (rc=1, no GPU error in its log): going on" | tee -a gpurun_out/steps.txt
    tail -n 5 "gpurun_out/$name.log"
    return 0
  fi
  if [ $rc -ne 0 ]; then
    echo "stopping after $name (rc=$rc)"
    tail -40 "gpurun_out/$name.log"
    exit $rc
  fi
  tail -n 2 "gpurun_out/$name.log"
}

expand() {
  case "$1" in
    roundend)
      echo "pytest_gpu|900|python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread"
      echo "smoke|200|python -u -c 'import __graft_entry__ as g; g.smoke()'"
      echo "bench|400|python -u bench.py";;
    trace)
      echo "trace|400|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5";;
    pmc)
      # one counter block per run (FETCH_SIZE, then WRITE_SIZE), per config
      for c in ${PMC_CONFIGS-1 2 3 4 5}; do
        case $c in 1) k=k_counter_key; n=10000;; 2) k=k_counter_quad2; n=10000000;;
                   3) k=k_tags; n=1000000;; 4) k=k_tags; n=1000000;; 5) k=k_gst_cols; n=4096;; esac
        echo "fetch$c|180|rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch$c -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --cpu-keys 0 --tune-rounds 0 --configs none"
        echo "write$c|180|rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write$c -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --cpu-keys 0 --tune-rounds 0 --configs none"
        echo "pmcj$c|60|python3 scripts/pmc_traffic.py gpurun_out/prof_fetch$c/run_counter_collection.csv gpurun_out/prof_write$c/run_counter_collection.csv $k $n $c gpurun_out/pmc/cfg$c.json"
      done
      # the one-pass GC kernel (segmented agn_prune_ops) on the cfg2 / cfg3 logs
      for c in ${PMC_GC_CONFIGS-2 3}; do
        case $c in 2) n=10000000;; 3) n=1000000;; esac
        echo "gcfetch$c|180|rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_gcfetch$c -o run -- python3 bench.py --config $c --gc --steps 1 --warmup 1 --cpu-keys 0 --tune-rounds 0 --configs none"
        echo "gcwrite$c|180|rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_gcwrite$c -o run -- python3 bench.py --config $c --gc --steps 1 --warmup 1 --cpu-keys 0 --tune-rounds 0 --configs none"
        echo "gcpmcj$c|60|python3 scripts/pmc_traffic.py gpurun_out/prof_gcfetch$c/run_counter_collection.csv gpurun_out/prof_gcwrite$c/run_counter_collection.csv k_prune_inplace $n gc gpurun_out/pmc/gc_cfg$c.json"
      done;;
    pmcsparse)
      # cfg2 with presence masks (bench.py --sparse MODE): the masked counter kernel
      for m in ${PMC_SPARSE-full mixed}; do
        echo "sfetch$m|180|rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_sfetch$m -o run -- python3 bench.py --config 2 --sparse $m --steps 3 --warmup 1 --cpu-keys 0 --tune-rounds 0 --configs none"
        echo "swrite$m|180|rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_swrite$m -o run -- python3 bench.py --config 2 --sparse $m --steps 3 --warmup 1 --cpu-keys 0 --tune-rounds 0 --configs none"
        case $m in mixed) sk=k_counter_key;; *) sk=k_counter_q8e2;; esac
        echo "spmcj$m|60|python3 scripts/pmc_traffic.py gpurun_out/prof_sfetch$m/run_counter_collection.csv gpurun_out/prof_swrite$m/run_counter_collection.csv $sk 10000000 2 gpurun_out/pmc/cfg2_sparse_$m.json"
      done;;
    pmcwarm)
      # warm cfg2 / cfg3 / cfg4 (bench.py --warm: k_counter_quad2 from the
      # cached base, k_tags from the cached states): the 3 warm steps'
      # launches, before the 4 of agn_read_cached's default dispatch (the
      # batched kernels: for counter_pn at D = 8 from 5M requests; its fused
      # form, timed after them, launches k_read6)
      for c in ${PMC_WARM-2 3 4}; do
        case $c in 2) k=k_counter_quad2; n=10000000; sel=tail:3:4;;
                   *) k=k_tags; n=1000000; sel=tail:3:4;; esac
        echo "wfetch$c|240|rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_wfetch$c -o run -- python3 bench.py --config $c --warm --steps 3 --warmup 1 --cpu-keys 0 --tune-rounds 0 --configs none"
        echo "wwrite$c|240|rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_wwrite$c -o run -- python3 bench.py --config $c --warm --steps 3 --warmup 1 --cpu-keys 0 --tune-rounds 0 --configs none"
        echo "wpmcj$c|60|python3 scripts/pmc_traffic.py gpurun_out/prof_wfetch$c/run_counter_collection.csv gpurun_out/prof_wwrite$c/run_counter_collection.csv $k $n $c gpurun_out/pmc/cfg${c}_warm.json $sel"
      done;;
    pmctail)
      # the engine-owned log's in-place GC (k_prune_tail) on the prefix-drop bench
      echo "tfetch|180|rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_tfetch -o run -- python3 scripts/bench_oplog_prune.py 2000000 64 3"
      echo "twrite|180|rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_twrite -o run -- python3 scripts/bench_oplog_prune.py 2000000 64 3"
      echo "tpmcj|60|python3 scripts/pmc_traffic.py gpurun_out/prof_tfetch/run_counter_collection.csv gpurun_out/prof_twrite/run_counter_collection.csv k_prune_tail 2000000 gc gpurun_out/pmc/oplog_prune_tail.json";;
    serve)
      # native read/6 serving (tools/serve_bench): 250k keys x 64 ops per
      # partition, D = 8, 20 read servers per partition; 1 and 8 partitions
      # (one batcher each); with writers (2000 updates/s per partition); and
      # a 2000-key hot set (cache hits, stores, GC)
      echo "serve1|150|./tools/serve_bench parts=1 threads=20 reads=20000"
      echo "serve8|150|./tools/serve_bench parts=8 threads=20 reads=5000"
      echo "serve8w|150|./tools/serve_bench parts=8 threads=20 reads=5000 wps=2000"
      echo "serve8h|150|./tools/serve_bench parts=8 threads=20 reads=5000 wps=2000 hot=2000"
      # the logs the Erlang NIF builds: presence masks on every clock, all 8
      # DCs interned, or 3 of 8 columns interned (partition width 8)
      echo "serve1s|150|./tools/serve_bench parts=1 threads=20 reads=20000 sparse=1"
      echo "serve8s|150|./tools/serve_bench parts=8 threads=20 reads=5000 sparse=1"
      echo "serve8sw|150|./tools/serve_bench parts=8 threads=20 reads=5000 wps=2000 sparse=1"
      echo "serve8s3|150|./tools/serve_bench parts=8 threads=20 reads=5000 sparse=1 present=3"
      echo "serve8sh|150|./tools/serve_bench parts=8 threads=20 reads=5000 wps=2000 hot=2000 sparse=1"
      # set_aw / register_mv partitions (states in the device cache's arena)
      echo "serve8set|150|./tools/serve_bench type=set parts=8 threads=20 reads=5000 wps=2000 sparse=1"
      echo "serve8reg|150|./tools/serve_bench type=register parts=8 threads=20 reads=5000 wps=2000 sparse=1"
      echo "serve8seth|150|./tools/serve_bench type=set parts=8 threads=20 reads=5000 wps=2000 hot=2000 sparse=1";;
    servetags)
      # set_aw / register_mv serving: the fused read (default) against the
      # kernel sequence (AGN_READ6=0), interleaved, dense and masked logs
      for r in 1 0; do
        echo "st1d_r$r|150|env AGN_READ6=$r ./tools/serve_bench type=set parts=1 threads=20 reads=20000"
        echo "st1s_r$r|150|env AGN_READ6=$r ./tools/serve_bench type=set parts=1 threads=20 reads=20000 sparse=1"
        echo "st8d_r$r|150|env AGN_READ6=$r ./tools/serve_bench type=set parts=8 threads=20 reads=5000 wps=2000"
        echo "st8s_r$r|150|env AGN_READ6=$r ./tools/serve_bench type=set parts=8 threads=20 reads=5000 wps=2000 sparse=1"
        echo "rg8s_r$r|150|env AGN_READ6=$r ./tools/serve_bench type=register parts=8 threads=20 reads=5000 wps=2000 sparse=1"
        echo "st8sh_r$r|150|env AGN_READ6=$r ./tools/serve_bench type=set parts=8 threads=20 reads=5000 wps=2000 hot=2000 sparse=1"
      done;;
    *) echo "$1";;
  esac
}

for spec in "$@"; do
  while IFS= read -r line; do
    [ -z "$line" ] && continue
    IFS='|' read -r name t cmd <<< "$line"
    run_step "$name" "$t" "$cmd"
  done < <(expand "$spec")
done
echo "all steps ok"
