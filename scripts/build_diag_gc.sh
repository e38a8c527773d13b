#!/bin/bash
# Diagnostic builds of the working tree's one-pass GC kernel (measurement
# only, never shipped): tools/libagn_diag_gc_<name>.so with one part of
# k_prune_inplace removed, to attribute cfg3's GC time
# (scripts/ab_prev_gc.py 3 name=tools/libagn_diag_gc_<name>.so ...; the
# outputs differ by design).  Reuses the working tree's other objects
# (antidote_amd/csrc/build/*.o: run make first), recompiles gc.hip only.
#   nofstore : kept entries' fields (op id, txid, tag, add token, rem_off)
#              loaded but not stored
#   nofload  : the kept entries' fields not loaded (nor their tokens)
#   notok    : no removal tokens moved (fields still loaded and stored)
#   norowst  : kept rows not stored
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
for V in ${DIAG_VARIANTS:-nofstore nofload notok norowst}; do
T=$(mktemp -d)
cp -r "$ROOT/antidote_amd" "$ROOT/include" "$T/"
python3 - "$T/antidote_amd/csrc/gc.hip" $V <<'PY'
import sys
p, v = sys.argv[1], sys.argv[2]
s = open(p).read()
def sub(old, new, count=1):
    global s
    assert s.count(old) == count, (v, old, s.count(old))
    s = s.replace(old, new)
if v == "nofstore":
    sub("""        if (head) {
            a.d_op_id[dst] = id;""", """        if (head && a.D == 0x5a5au) {
            a.d_op_id[dst] = id;""")
elif v == "nofload":
    sub("if (late && !have && kp && sub == 0) load_fields();", "")
elif v == "notok":
    sub("        if (!head) rl_ = 0;\n", "        rl_ = 0;\n")
elif v == "norowst":
    sub("""        } else if (kp) {
            if constexpr (FULL) {
                u64x2 *q = reinterpret_cast<u64x2 *>(a.d_oc + dst * D + (uint32_t)d0);""",
        """        } else if (kp && a.D == 0x5a5au) {
            if constexpr (FULL) {
                u64x2 *q = reinterpret_cast<u64x2 *>(a.d_oc + dst * D + (uint32_t)d0);""")
open(p, "w").write(s)
PY
cd "$T/antidote_amd/csrc"
rm -f build/gc.o
make -s build/gc.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-Bsymbolic -o "$ROOT/tools/libagn_diag_gc_$V.so" \
    build/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
cd "$ROOT"
rm -rf "$T"
echo "built tools/libagn_diag_gc_$V.so"
done
