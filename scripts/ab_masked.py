"""A/B of the masked counter kernel (presence masks, uniform keys) against the
dense one on cfg2 in one process, variants interleaved: which of the masked
batch's extra inputs / outputs costs what, on uniform keys and on mixed ones
(bench.py --sparse mixed masks).  Round 3 also timed the register budget of
8 waves per SIMD for cold masked batches ("_w8" variants: 8.51 vs 8.49 ms,
mixed 9.57 vs 9.46; profiles/r03/ab_masked_w8.log) -- not kept.

Round 4: each variant also carries environment knobs (AGN_COUNTER_EARLY=0:
k_counter_key, the prologue with every scalar load before the rows; default:
k_counter_q8e + k_counter_q8m over the keys whose entries differ, chunk 0's
rows issued right after the segment metadata and the key's DC set;
AGN_Q8E_KM=1: the DC set loaded with the metadata instead of under the
chunk) and agn_read.hints
(AGN_HINT_CT_FLAG / AGN_HINT_R_FULL).  Every variant's results (value, hole,
LastOpCt + its mask, count, flags) are compared with its input class's first
variant.

  python scripts/ab_masked.py [rounds]
"""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from antidote_amd._lib import env_changed  # noqa: E402

HINTS = 0x1 | 0x2  # AGN_HINT_R_FULL | AGN_HINT_CT_FLAG
# name: (inputs, env, hints)
VARIANTS = {
    "dense": ("dense", {}, 0),
    "masked_old": ("masked", {"AGN_COUNTER_EARLY": "0"}, 0),
    "masked": ("masked", {}, 0),
    "masked_km1": ("masked", {"AGN_Q8E_KM": "1"}, 0),
    "masked_ctflag": ("masked", {}, 0x2),
    "masked_hints": ("masked", {}, HINTS),
    "mixed_old": ("mixed", {"AGN_COUNTER_EARLY": "0"}, 0),
    "mixed": ("mixed", {}, 0),
    "mixed_km1": ("mixed", {"AGN_Q8E_KM": "1"}, 0),
    "mixed_hint": ("mixed", {}, 0x4),   # AGN_HINT_MIXED: k_counter_key
    "masked_two": ("masked", {"AGN_Q8E_TWO": "1"}, 0x2),  # warm: k_counter_q8e2
    # warm masked batches default to k_counter_q8e2 (round 5); one request
    # per wave (k_counter_q8e) with the bench's hints
    "masked_one": ("masked", {"AGN_Q8E_TWO": "0"}, HINTS),
    # round 5: the dense kernel one request per wave (k_counter_key quad rows;
    # warm dense batches default to two per wave, k_counter_quad2), and the
    # masked batch through k_counter_quad2's MSK form
    "dense_q1": ("dense", {"AGN_COUNTER_VARIANT": "2"}, 0),
    "masked_quad2": ("masked", {"AGN_COUNTER_VARIANT": "3"}, HINTS),
    "masked_old_hints": ("masked", {"AGN_COUNTER_EARLY": "0"}, HINTS),
    # round 6: block orders (identity by default for the masked forms)
    "masked_x1": ("masked", {"AGN_XCD_REMAP": "1"}, 0),
    "masked_c64": ("masked", {"AGN_XCD_CHUNK": "64"}, 0),
    "masked_two_x1": ("masked", {"AGN_Q8E_TWO": "1", "AGN_XCD_REMAP": "1"}, 0x2),
    "masked_two_c64": ("masked", {"AGN_Q8E_TWO": "1", "AGN_XCD_CHUNK": "64"}, 0x2),
    "masked_hints_x1": ("masked", {"AGN_XCD_REMAP": "1"}, HINTS),
    "masked_hints_c64": ("masked", {"AGN_XCD_CHUNK": "64"}, HINTS),
    # cold batches two requests per wave (k_counter_q8e2's cold form)
    "masked_cold2": ("masked", {"AGN_Q8E_TWO": "2"}, 0),
    "masked_hints_cold2": ("masked", {"AGN_Q8E_TWO": "2"}, HINTS),
    "mixed_cold2": ("mixed", {"AGN_Q8E_TWO": "2"}, 0),
}
KNOBS = ("AGN_COUNTER_EARLY", "AGN_Q8E_KM", "AGN_Q8E_TWO", "AGN_COUNTER_VARIANT", "AGN_XCD_REMAP",
         "AGN_XCD_CHUNK")


def main():
    import torch
    from antidote_amd import _abi
    from antidote_amd.engine import Engine
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    only = [x for x in os.environ.get("AB_ONLY", "").split(",") if x]
    torch.cuda.set_device(0)
    eng = Engine(0)
    st = torch.cuda.current_stream()
    sp = st.cuda_stream
    K, N, D = 10_000_000, 64, 8
    g = _abi.AgnGenCfg(crdt_type=1, n_dcs=D, n_keys=K, ops_per_key=N, n_elems=0,
                       seed=20250113, key_base=0, key_stride=1, warm=int(os.environ.get("WARM", "0")))
    dl, dr = eng.gen_dev(g)
    ocm = torch.full((K * N,), 255, dtype=torch.int64, device="cuda")
    rm = torch.full((K,), 255, dtype=torch.int64, device="cuda")
    from bench import presence_masks
    ocm_x, _ = presence_masks("mixed", D, K * N, K, torch=torch)
    kb, kbx = eng.empty(8 * K), eng.empty(8 * K)
    res = {"dense": eng.alloc_result(K, D, sparse=False),
           "masked": eng.alloc_result(K, D, sparse=True),
           "mixed": eng.alloc_result(K, D, sparse=True)}

    def structs(inputs, hints):
        ls, rs = _abi.AgnLog(), _abi.AgnRead()
        C.memmove(C.addressof(ls), C.addressof(dl), C.sizeof(ls))
        C.memmove(C.addressof(rs), C.addressof(dr), C.sizeof(rs))
        if inputs != "dense":
            ls.oc_mask = (ocm if inputs == "masked" else ocm_x).data_ptr()
            ls.key_mask = (kb if inputs == "masked" else kbx).ptr
            rs.R_mask = rm.data_ptr()
        rs.hints = hints
        return ls, rs
    names = [n for n in VARIANTS if not only or n in only]
    args = {n: structs(VARIANTS[n][0], VARIANTS[n][2]) for n in names}
    for inputs, buf in (("masked", kb), ("mixed", kbx)):
        ls, _ = structs(inputs, 0)
        assert eng.lib.agn_log_index_masks(eng.ctx, C.byref(ls), buf.ptr, sp) == 0

    def setenv(env):
        for k in KNOBS:
            if k in env:
                os.environ[k] = env[k]
                env_changed()
            else:
                os.environ.pop(k, None)
                env_changed()
    ms = {n: [] for n in names}
    ref, same = {}, {}
    for r in range(rounds + 1):
        for n in (names if r % 2 == 0 else names[::-1]):
            inputs, env, _ = VARIANTS[n]
            ls, rs = args[n]
            setenv(env)
            b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            b.record(st)
            eng.materialize(ls, rs, res[inputs], stream=sp)
            e.record(st)
            torch.cuda.synchronize()
            if r:
                ms[n].append(b.elapsed_time(e))
            if r == 0:  # results of every variant vs its input class's first
                got = eng.fetch_result(res[inputs])
                key = "dense" if inputs in ("dense", "masked") else "mixed"
                fields = ("value", "hole", "lastct", "count", "flags") + \
                    (("lastct_mask",) if inputs != "dense" else ())
                if key not in ref:
                    ref[key] = got
                    same[n] = True
                else:
                    same[n] = all(np.array_equal(getattr(got, f), getattr(ref[key], f))
                                  for f in fields if getattr(ref[key], f) is not None)
                if inputs == "masked" and "masked" not in ref:
                    ref["masked"] = got
                if inputs == "masked":
                    same[n] = same[n] and np.array_equal(got.lastct_mask, ref["masked"].lastct_mask)
    setenv({})
    med = {n: float(np.median(x)) for n, x in ms.items()}
    base = med.get("dense")
    print(json.dumps({"warm": int(os.environ.get("WARM", "0")),
                      "ms_median": med,
                      "vs_dense": {n: (v / base if base else None) for n, v in med.items()},
                      "results_equal": same}), flush=True)
    dl.oc_mask = dr.R_mask = None
    eng.free_gen(dl, dr)
    eng.close()


if __name__ == "__main__":
    main()
