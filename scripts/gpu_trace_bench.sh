# rocprofv3 kernel-trace stats of the bench command itself (one process per
# config): the bench line's HIP-event kernel_ms and rocprof's average duration
# of the same kernel come from the same run, so they must agree.
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
for c in 2 3 4; do
  step tb$c 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tb$c -o run -- python3 bench.py --config $c
done
tail -qn1 gpurun_out/tb2.log gpurun_out/tb3.log gpurun_out/tb4.log
