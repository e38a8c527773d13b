"""SURVEY.md §8(f) rank-4 row at bulk size: the causal-dependency check of
inter_dc_dep_vnode:try_store/2 (agn_dep_check) over n transactions against
P partition clocks, dense and presence-masked clocks, the current library
against tools/libagn_prev.so (scripts/build_prev.sh) in one process,
interleaved; the outputs must be identical.  Roofline: algorithmic bytes per
launch = n (8 D deps + 4 origin + 4 part + 1 flag [+ 8 W deps mask]) + the
P partition clocks, over the median kernel time (HIP events on the launch
stream).

  python scripts/bench_dep_check.py [n=10000000] [D=8,64] [P=64]
"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from antidote_amd import _abi  # noqa: E402
from antidote_amd.engine import Engine  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
DS = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "8,64").split(",")]
P = int(sys.argv[3]) if len(sys.argv) > 3 else 64
PEAK = 8000.0  # GB/s

eng = Engine(0)
prev = C.CDLL(os.path.join(ROOT, "tools", "libagn_prev.so"), mode=os.RTLD_LOCAL)
_abi.bind(prev, {k: v for k, v in _abi.PROTOTYPES.items() if hasattr(prev, k)})
pctx = C.c_void_p()
assert prev.agn_open(0, C.byref(pctx)) == 0
sp = torch.cuda.current_stream().cuda_stream


def case(D, sparse, seed):
    rng = np.random.default_rng(seed)
    W = (D + 63) // 64
    pc = rng.integers(1000, 2000, (P, D)).astype(np.uint64)
    part = rng.integers(0, P, N).astype(np.uint32)
    origin = rng.integers(0, D, N).astype(np.uint32)
    deps = (pc[part] - rng.integers(0, 40, (N, D))).astype(np.uint64)
    ahead = rng.random(N) < 0.5
    col = rng.integers(0, D, N)
    deps[ahead, col[ahead]] = pc[part[ahead], col[ahead]] + np.uint64(1)
    dm = pm = None
    if sparse:
        full = np.uint64((1 << D) - 1) if D < 64 else np.uint64(0xFFFFFFFFFFFFFFFF)
        pm = np.full((P, W), full, np.uint64)
        dm = np.full((N, W), full, np.uint64)
        drop = rng.random(N) < 0.2  # a fifth of the snapshots miss one DC
        dc = rng.integers(0, D, N)
        dm[drop, dc[drop] >> 6] &= ~(np.uint64(1) << (dc[drop] & 63).astype(np.uint64))
    return deps, dm, origin, part, pc, pm


out = {}
for D in DS:
    for sparse in (False, True):
        arrs = case(D, sparse, D * 7 + sparse)
        bufs = [eng.upload(x) if x is not None else None for x in arrs]
        ptrs = [b.ptr if b is not None else None for b in bufs]
        oks = {"cur": eng.empty(N), "prev": eng.empty(N)}

        def run(v):
            lib, ctx = (eng.lib, eng.ctx) if v == "cur" else (prev, pctx)
            rc = lib.agn_dep_check(ctx, D, N, ptrs[0], ptrs[1], ptrs[2], ptrs[3], P, ptrs[4],
                                   ptrs[5], oks[v].ptr, sp)
            assert rc == 0

        times = {"cur": [], "prev": []}
        for rnd in range(12):
            for v in (("cur", "prev") if rnd % 2 == 0 else ("prev", "cur")):
                b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                b.record()
                run(v)
                e.record()
                torch.cuda.synchronize()
                if rnd >= 2:
                    times[v].append(b.elapsed_time(e))
        W = (D + 63) // 64
        alg = N * (8 * D + 4 + 4 + 1 + (8 * W if sparse else 0)) + P * (8 * D + (8 * W if sparse else 0))
        same = np.array_equal(eng.download(oks["cur"], np.uint8, (N,)),
                              eng.download(oks["prev"], np.uint8, (N,)))
        applicable = float(eng.download(oks["cur"], np.uint8, (N,)).mean())
        rec = {"n_txn": N, "n_dcs": D, "n_parts": P, "masked": sparse, "identical": same,
               "applicable_frac": applicable, "algorithmic_bytes": alg}
        for v, t in times.items():
            ms = float(np.median(t))
            rec[v] = {"ms": ms, "txn_per_s": N / (ms * 1e-3), "GB_s": alg / ms / 1e6,
                      "frac_of_8TBs": alg / ms / 1e6 / PEAK}
        out[f"D{D}{'_masked' if sparse else ''}"] = rec
        print(json.dumps(rec), flush=True)
        for b in bufs + list(oks.values()):
            if b is not None:
                b.free()
