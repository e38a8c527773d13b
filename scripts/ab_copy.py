"""Read+write probe A/B (tools/copyprobe_ab.hip): which idiom streams a copy /
the GC's 3:4 write mix fastest on this box.  16 GiB source, 16 GiB destination,
variants interleaved in one process; GB/s counts bytes read + bytes written.

  python scripts/ab_copy.py [variant ...]      (AGN_COPY_WQ=3|4, default both)
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = C.CDLL(os.path.join(ROOT, "tools", "libagn_copyprobe_ab.so"))
lib.agn_copy_variant.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, C.c_void_p]
NB = int(os.environ.get("AGN_PROBE_GIB", "16")) << 30
src = torch.empty(NB, dtype=torch.uint8, device="cuda")
src.random_(0, 256)
dst = torch.empty(NB, dtype=torch.uint8, device="cuda")
sp = torch.cuda.current_stream().cuda_stream
names = {0: "oneshot 4KiB", 1: "oneshot nt ld+st", 2: "oneshot nt st", 3: "glds ld, st",
         4: "oneshot 8KiB", 5: "gridstride", 6: "oneshot wpb4", 7: "oneshot in place",
         8: "glds in place"}
V = [int(x) for x in sys.argv[1:]] or sorted(names)
WQ = [int(os.environ["AGN_COPY_WQ"])] if os.environ.get("AGN_COPY_WQ") else [4, 3]
for wq in WQ:
    t = {v: [] for v in V}
    for rnd in range(int(os.environ.get("AGN_PROBE_ROUNDS", "7"))):
        for v in V:
            b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            b.record()
            assert lib.agn_copy_variant(v, src.data_ptr(), dst.data_ptr(), NB, wq, sp) == 0
            e.record()
            torch.cuda.synchronize()
            if rnd >= 2:
                t[v].append(b.elapsed_time(e))
    moved = NB + NB * wq // 4
    for v in V:
        ms = float(np.median(t[v]))
        print(f"wq{wq} v{v} {names[v]:20s} {ms:.3f} ms  {moved / ms / 1e6:.0f} GB/s "
              f"(best {moved / min(t[v]) / 1e6:.0f})", flush=True)
