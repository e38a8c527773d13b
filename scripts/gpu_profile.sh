# Round profile: bench lines for cfg2/3/4 (+GST), rocprofv3 kernel-trace stats
# and FETCH_SIZE / WRITE_SIZE passes (one counter per run) for each config,
# plus a FETCH_SIZE calibration of the 16-byte and 4-byte LDS-DMA widths.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.txt
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -20 "gpurun_out/$name.log"; exit $rc; fi
  return 0
}
: > gpurun_out/steps.txt
export AGN_PROBE_GIB=4 AGN_PROBE_ROUNDS=3
step calib 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_calib -o run -- python3 scripts/ab_probe.py 4 10
unset AGN_PROBE_GIB AGN_PROBE_ROUNDS
step bench2 400 python -u bench.py --config 2 --gst
step bench3 400 python -u bench.py --config 3
step bench4 400 python -u bench.py --config 4
for c in 2 3 4; do
  step trace$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace$c -o run -- python3 bench.py --config $c --steps 10 --warmup 2 --cpu-keys 0
  step fetch$c 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch$c -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --cpu-keys 0
  step write$c 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write$c -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --cpu-keys 0
done
tail -qn1 gpurun_out/bench2.log gpurun_out/bench3.log gpurun_out/bench4.log
