"""Where a small batch's step goes (cfg1: 10k keys x 100 ops, D = 3): the
host issue cost of one agn_materialize call through ctypes, with and without
per-step HIP events, against the kernel's own time.

Each variant issues N launches back to back on one stream and reports the
wall time per launch once the stream drained (host-bound when above the
kernel time) and the host-side issue time alone (the loop without waiting).

  python scripts/launch_overhead.py [N]
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    from antidote_amd import _abi
    from antidote_amd.engine import Engine
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    torch.cuda.set_device(0)
    eng = Engine(0)
    st = torch.cuda.current_stream()
    sp = st.cuda_stream
    g = _abi.AgnGenCfg(crdt_type=1, n_dcs=3, n_keys=10_000, ops_per_key=100, n_elems=0,
                       seed=20250112, key_base=0, key_stride=1, warm=0)
    dl, dr = eng.gen_dev(g)
    res = eng.alloc_result(10_000, 3, sparse=False)
    lib = eng.lib
    ls, rs, os_ = C.byref(dl), C.byref(dr), C.byref(res.struct)
    fn, ctx = lib.agn_materialize, eng.ctx

    def wrapper():
        eng.materialize(dl, dr, res, stream=sp)

    def prebound():
        if fn(ctx, ls, rs, os_, sp):
            raise RuntimeError("agn_materialize")

    out = {}
    for name, call, events in (("wrapper", wrapper, False), ("prebound", prebound, False),
                               ("wrapper+events", wrapper, True),
                               ("prebound+events", prebound, True)):
        for _ in range(200):
            call()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(N)] if events else None
        t0 = time.perf_counter()
        for i in range(N):
            if events:
                ev[i][0].record(st)
            call()
            if events:
                ev[i][1].record(st)
        t_issue = time.perf_counter() - t0
        torch.cuda.synchronize()
        t_all = time.perf_counter() - t0
        r = {"us_per_step": t_all / N * 1e6, "host_issue_us": t_issue / N * 1e6}
        if events:
            r["kernel_us"] = float(np.mean([a.elapsed_time(b) for a, b in ev])) * 1e3
        out[name] = r
    # the kernel alone, one event pair around N back-to-back launches
    b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    b.record(st)
    for _ in range(N):
        prebound()
    e.record(st)
    torch.cuda.synchronize()
    out["stream_us_per_launch"] = b.elapsed_time(e) * 1e3 / N
    print(json.dumps(out), flush=True)
    eng.free_gen(dl, dr)
    eng.close()


if __name__ == "__main__":
    main()
