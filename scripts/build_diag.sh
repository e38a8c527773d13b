#!/bin/bash
# Diagnostic builds of the working tree's counter kernel (measurement only,
# never shipped): tools/libagn_diag_<name>.so with one cost removed, to
# attribute the gap between the cfg2 kernel and the read-ceiling probe.
#   noeff   : no effect loads (8 B/op less)
#   fewwr   : only value + hole written (LastOpCt/count/flags/err folded in)
#   nometa  : key_off/len not loaded (cfg2 shape: off = key*64, n = 64)
#   rec     : outputs as one 128 B record per key (one full line, 8 lanes x
#             16 B) into the buffer passed as err_pos (scripts/ab_prev.py)
#   ntwr    : SoA outputs through non-temporal stores
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
for V in ${DIAG_VARIANTS:-noeff fewwr nometa}; do
T=$(mktemp -d)
cp -r "$ROOT/antidote_amd" "$ROOT/include" "$T/"
rm -rf "$T/antidote_amd/csrc/build"
python3 - "$T/antidote_amd/csrc/mat_counter_dense.hip" $V <<'PY'
import sys
p, v = sys.argv[1], sys.argv[2]
s = open(p).read()
if v == "noeff":
    old = "        const int64_t ev = eff[e];\n"
    assert s.count(old) == 1
    s = s.replace(old, "        const int64_t ev = (int64_t)(e & 7);\n")
elif v == "fewwr":
    old = "    if (g == 0 && c < D) o_lastct[i * D + (uint64_t)c] = ct_ign ? 0ull : m;\n"
    assert s.count(old) == 2
    s = s.replace(old, "    const uint64_t mm = ballot(m == 12345ull) ^ (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)m);\n", 1)
    old = """        o_hole[i] = hole;
        o_count[i] = cnt;
        o_flags[i] = fl;
        o_err[i] = first_err >= 0 ? (uint32_t)(off + (uint64_t)first_err) : 0xffffffffu;"""
    assert s.count(old) == 1
    s = s.replace(old, """        o_hole[i] = hole ^ (int64_t)mm ^ (int64_t)cnt ^ ((int64_t)fl << 40) ^ (first_err << 20);""")
elif v == "rec":
    old = """    if (g == 0 && c < D) o_lastct[i * D + (uint64_t)c] = ct_ign ? 0ull : m;
    if (lane == 0) {
        // NewLastOp = id(oldest excluded) - 1, else get_first_id (:49-63)
        const int64_t hole = first_excl >= 0 ? hid - 1 : hid;
        uint32_t fl = 0;
        if (cnt) fl |= AGN_F_NEWSS;
        if (ct_ign) fl |= AGN_F_CT_IGNORE;
        if (first_err >= 0) fl |= AGN_F_ERR_UNEXPECTED;
        o_value[i] = (int64_t)((uint64_t)base + (uint64_t)total);
        o_hole[i] = hole;
        o_count[i] = cnt;
        o_flags[i] = fl;
        o_err[i] = first_err >= 0 ? (uint32_t)(off + (uint64_t)first_err) : 0xffffffffu;
    }"""
    assert s.count(old) == 1
    s = s.replace(old, """    {
        const int64_t hole = first_excl >= 0 ? hid - 1 : hid;
        uint32_t fl = 0;
        if (cnt) fl |= AGN_F_NEWSS;
        if (ct_ign) fl |= AGN_F_CT_IGNORE;
        if (first_err >= 0) fl |= AGN_F_ERR_UNEXPECTED;
        const uint64_t mv = ct_ign ? 0ull : m;
        const int src = (lane & 3) * 2;
        auto sh = [](uint64_t v, int l) {
            return ((uint64_t)(uint32_t)__shfl((int)(v >> 32), l, 64) << 32) | (uint32_t)__shfl((int)(uint32_t)v, l, 64);
        };
        uint64_t a0 = sh(mv, src), a1 = sh(mv, src + 1);
        if (src >= D) a0 = 0;
        if (src + 1 >= D) a1 = 0;
        uint64_t x0 = 0, x1 = 0;
        if (lane < 4) { x0 = a0; x1 = a1; }
        else if (lane == 4) { x0 = (uint64_t)base + (uint64_t)total; x1 = (uint64_t)hole; }
        else if (lane == 5) { x0 = (uint64_t)cnt | ((uint64_t)fl << 32);
                              x1 = first_err >= 0 ? (off + (uint64_t)first_err) : 0xffffffffull; }
        if (lane < 8) reinterpret_cast<u64x2 *>(o_err)[i * 8 + (uint64_t)lane] = u64x2{x0, x1};
    }""")
elif v == "ntwr":
    for a, b in (("o_lastct[i * D + (uint64_t)c] = ct_ign ? 0ull : m;", "__builtin_nontemporal_store(ct_ign ? 0ull : m, o_lastct + i * D + (uint64_t)c);"),
                 ("o_value[i] = (int64_t)((uint64_t)base + (uint64_t)total);", "__builtin_nontemporal_store((int64_t)((uint64_t)base + (uint64_t)total), o_value + i);"),
                 ("o_hole[i] = hole;", "__builtin_nontemporal_store(hole, o_hole + i);"),
                 ("o_count[i] = cnt;", "__builtin_nontemporal_store(cnt, o_count + i);"),
                 ("o_flags[i] = fl;", "__builtin_nontemporal_store(fl, o_flags + i);"),
                 ("o_err[i] = first_err >= 0 ? (uint32_t)(off + (uint64_t)first_err) : 0xffffffffu;", "__builtin_nontemporal_store(first_err >= 0 ? (uint32_t)(off + (uint64_t)first_err) : 0xffffffffu, o_err + i);")):
        assert a in s, a
        s = s.replace(a, b, 1)
elif v == "nometa":
    old = "    const KeyMeta km = key_meta(key, key_off, key_len, key_id0);\n    const uint64_t off = km.off, n = km.n;\n    const uint32_t id0 = km.id0;"
    assert s.count(old) == 1
    s = s.replace(old, "    const uint64_t off = key * 64u, n = 64u;\n    const uint32_t id0 = 1u;")
open(p, "w").write(s)
PY
cd "$T/antidote_amd/csrc"
make -s -j8 build/api.o build/mat_counter.o build/mat_counter_dense.o build/mat_tags.o build/gst.o \
    build/gc.o build/cache.o build/ingest.o build/oplog.o build/batcher.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-Bsymbolic -o "$ROOT/tools/libagn_diag_$V.so" \
    build/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
cd "$ROOT"; rm -rf "$T"
echo "built tools/libagn_diag_$V.so"
done
