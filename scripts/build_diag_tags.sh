#!/bin/bash
# Diagnostic builds of the working tree's set/register kernel (measurement
# only, never shipped): tools/libagn_diag_tags_<name>.so with one phase of
# k_tags removed, to attribute cfg3's time (scripts/ab_prev.py 3
# name=tools/libagn_diag_tags_<name>.so ...; results differ by design).
#   norem    : no removal phase (no rem_tok loads, no token walk)
#   noadd    : no candidates (no adds kept: the LDS table, its removal
#              matches, the compaction, sort and state output all empty)
#   nosort   : the live state written unsorted (no bitonic sort)
#   nofilter : the row verdicts from one ballot (the rows are still loaded
#              and consumed), no compares / group folds
#   norows   : no row loads (synthetic rows from the lane id)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
for V in ${DIAG_VARIANTS:-norem noadd nosort nofilter norows}; do
T=$(mktemp -d)
cp -r "$ROOT/antidote_amd" "$ROOT/include" "$T/"
rm -rf "$T/antidote_amd/csrc/build"
python3 - "$T/antidote_amd/csrc/mat_tags.hip" $V <<'PY'
import sys
p, v = sys.argv[1], sys.argv[2]
s = open(p).read()
def sub(old, new, count=1):
    global s
    assert s.count(old) == count, (v, old, s.count(old))
    s = s.replace(old, new)
if v == "norem":
    sub("const uint32_t K1 = __builtin_amdgcn_readlane(cs.ro1, nvalid - 1);",
        "const uint32_t K1 = K0 + 0u * __builtin_amdgcn_readlane(cs.ro1, nvalid - 1);")
elif v == "noadd":
    sub("const bool adds = incl_e && cs.add != 0ull;", "const bool adds = incl_e && cs.add == 0x5a5a5a5a5a5aull;")
elif v == "nosort":
    sub("                bitonic<SET, CAP>(L, n_live);\n", "")
elif v == "nofilter":
    sub("""                    const uint64_t bad = group_any<P>(ballot(o0.x > rA || o0.y > rB)) |
                                         (group_any<P>(ballot(o1.x > rA || o1.y > rB)) << OPH);""",
        """                    const uint64_t bad = ballot((o0.x ^ o1.y) == 0x5a5a5a5a5aull && rA != 0ull) & 1ull;""")
elif v == "norows":
    sub("""                cx0 = __builtin_nontemporal_load(rows16 + (u < ue ? u : ue));
                cx1 = __builtin_nontemporal_load(rows16 + (u + AGN_WAVE < ue ? u + AGN_WAVE : ue));""",
        """                cx0 = u64x2{u & 7ull, u & 3ull};
                cx1 = u64x2{(u + 1ull) & 7ull, u & 1ull};""")
else:
    raise SystemExit("unknown variant " + v)
open(p, "w").write(s)
PY
cd "$T/antidote_amd/csrc"
make -s -j8 $(ls *.hip | sed 's/\.hip$/.o/; s/^/build\//')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-Bsymbolic -o "$ROOT/tools/libagn_diag_tags_$V.so" \
    build/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
cd "$ROOT"; rm -rf "$T"
echo "built tools/libagn_diag_tags_$V.so"
done
