# Attribution of the cfg2 counter kernel's gap to the read ceiling (diagnostic builds, scripts/build_diag.sh).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
timeout -k 10 300 python -u scripts/ab_prev.py 2 ${AB_LIBS:-fewwr=tools/libagn_diag_fewwr.so rec=tools/libagn_diag_rec.so ntwr=tools/libagn_diag_ntwr.so} > gpurun_out/ab_diag_$r.log 2>&1 || { echo "ab rc=$?"; tail gpurun_out/ab_diag_$r.log; exit 1; }
grep cfg gpurun_out/ab_diag_$r.log
done
