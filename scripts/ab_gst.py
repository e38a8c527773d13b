"""A/B of the column-resident GST kernel (k_gst_cols, agn_gst_min) on the
cfg5 batched shape (E = 256 epochs x P = 4096 partitions x D = 256), variants
alternated in one process: AGN_GST_BLOCKS (target blocks) x AGN_GST_UNROLL
(rows in flight per thread) x AGN_GST_NT (non-temporal loads).  Every variant's output must be identical.

  python scripts/ab_gst.py [rounds]
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from antidote_amd._lib import env_changed  # noqa: E402


def main():
    import torch
    from antidote_amd.engine import Engine
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    D, P, E = 256, 4096, 256
    torch.cuda.init()
    eng = Engine(0)
    sp = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda")
    g.manual_seed(20250116)
    clocks = torch.randint(0, 10 ** 9, (E, P, D), device="cuda", dtype=torch.int64,
                           generator=g) + 1_700_000_000_000_000
    out = torch.empty((E, D + 1), device="cuda", dtype=torch.int64)
    nbytes = E * P * D * 8 + E * (D + 1) * 8
    variants = [(f"b{b}_u{u}_nt{nt}", b, u, nt) for b in ("1024", "2048", "4096")
                for u in ("4", "8") for nt in ("0", "1")]
    ms = {v[0]: [] for v in variants}
    ref = None
    for r in range(rounds):
        for name, b, u, nt in (variants if r % 2 == 0 else variants[::-1]):
            os.environ["AGN_GST_BLOCKS"], os.environ["AGN_GST_UNROLL"] = b, u
            env_changed()
            os.environ["AGN_GST_NT"] = nt
            env_changed()
            eng.gst_min(D, P, E, clocks.data_ptr(), None, out.data_ptr(), sp)
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            assert torch.equal(out, ref), name
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                eng.gst_min(D, P, E, clocks.data_ptr(), None, out.data_ptr(), sp)
            e.record()
            torch.cuda.synchronize()
            ms[name].append(s.elapsed_time(e) / 5)
    med = {k: float(np.median(v)) for k, v in ms.items()}
    print(json.dumps({"shape": [E, P, D], "ms_median": med,
                      "GBps": {k: nbytes / (v * 1e-3) / 1e9 for k, v in med.items()},
                      "ms_all": ms}), flush=True)


if __name__ == "__main__":
    main()
