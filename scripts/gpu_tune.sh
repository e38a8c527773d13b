# agn_tune: parity tests, then the default bench (tuned) and a forced-VGPR bench.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.txt
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -40 "gpurun_out/$name.log"; exit $rc; fi
  return 0
}
: > gpurun_out/steps.txt
step tune_tests 300 python -u -m pytest tests/test_gpu_parity.py tests/test_id_index.py -m gpu -x -q --timeout 120 --timeout-method thread
tail -2 gpurun_out/tune_tests.log
step bench_tuned 300 python -u bench.py --cpu-keys 0
step bench_vgpr 300 env AGN_COUNTER_GLDS=0 python -u bench.py --cpu-keys 0
step bench_glds 300 env AGN_COUNTER_GLDS=1 python -u bench.py --cpu-keys 0
python - <<'PY'
import json
for n in ("bench_tuned", "bench_vgpr", "bench_glds"):
    j = json.loads([l for l in open(f"gpurun_out/{n}.log") if l.startswith('{"metric"')][-1])
    print(n, round(j["roofline"]["kernel_ms"], 3), round(j["roofline"]["frac"], 3), j.get("kernel_variant"))
PY
