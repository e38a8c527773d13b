"""A/B of the masked counter kernel (presence masks, uniform keys) against the
dense one on cfg2 in one process, variants interleaved: which of the masked
batch's extra inputs / outputs costs what, on uniform keys and on mixed ones
(bench.py --sparse mixed masks).  Round 3 also timed the register budget of
8 waves per SIMD for cold masked batches ("_w8" variants: 8.51 vs 8.49 ms,
mixed 9.57 vs 9.46; profiles/r03/ab_masked_w8.log) -- not kept.

  python scripts/ab_masked.py [rounds]
"""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    from antidote_amd import _abi
    from antidote_amd.engine import Engine
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
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
    kbx = eng.empty(8 * K)
    res_d = eng.alloc_result(K, D, sparse=False)
    res_s = eng.alloc_result(K, D, sparse=True)
    res_x = eng.alloc_result(K, D, sparse=True)
    kb = eng.empty(8 * K)

    def variant(name):
        ls, rs = _abi.AgnLog(), _abi.AgnRead()
        C.memmove(C.addressof(ls), C.addressof(dl), C.sizeof(ls))
        C.memmove(C.addressof(rs), C.addressof(dr), C.sizeof(rs))
        res = res_d
        if name != "dense":
            ls.oc_mask = ocm.data_ptr()
            ls.key_mask = kb.ptr
            rs.R_mask = rm.data_ptr()
            res = res_s
        if name == "masked_no_out_mask":
            res = res_d
        if name == "masked_no_R_mask":
            rs.R_mask = None
        if name.startswith("mixed"):
            ls.oc_mask = ocm_x.data_ptr()
            ls.key_mask = kbx.ptr
            res = res_x
        if name == "out_mask_only":
            ls.oc_mask = None
            ls.key_mask = None
            rs.R_mask = None
            res = res_s
        return ls, rs, res
    names = ["dense", "masked", "masked_no_out_mask", "masked_no_R_mask", "out_mask_only",
             "mixed"]
    args = {n: variant(n) for n in names}
    check = eng.lib.agn_log_index_masks(eng.ctx, C.byref(args["masked"][0]), kb.ptr, sp)
    assert check == 0
    check = eng.lib.agn_log_index_masks(eng.ctx, C.byref(args["mixed"][0]), kbx.ptr, sp)
    assert check == 0
    ms = {n: [] for n in names}
    for r in range(rounds + 1):
        for n in (names if r % 2 == 0 else names[::-1]):
            ls, rs, res = args[n]
            b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            b.record(st)
            eng.materialize(ls, rs, res, stream=sp)
            e.record(st)
            torch.cuda.synchronize()
            if r:
                ms[n].append(b.elapsed_time(e))
    v = {n: eng.download(args[n][2].bufs["value"], np.int64, (K,)) for n in names}
    # uniform masks give the dense values; the mixed log's own pair must agree
    same = {n: bool(np.array_equal(v[n], v["mixed" if n.startswith("mixed") else "dense"]))
            for n in names}
    print(json.dumps({"warm": int(os.environ.get("WARM", "0")),
                      "variant": os.environ.get("AGN_COUNTER_VARIANT", "default"),
                      "ms_median": {n: float(np.median(x)) for n, x in ms.items()},
                      "values_equal_dense": same}), flush=True)
    dl.oc_mask = dr.R_mask = None
    eng.free_gen(dl, dr)
    eng.close()


if __name__ == "__main__":
    main()
