"""Read-path probe A/B (tools/bwprobe_ab.hip): which streaming idiom reads HBM
fastest on this box.  32 GiB buffer, variants interleaved in one process."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = C.CDLL(os.path.join(ROOT, "tools", "libagn_probe_ab.so"))
lib.agn_probe_variant.argtypes = [C.c_int, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]
NB = int(os.environ.get("AGN_PROBE_GIB", "32")) << 30
buf = torch.empty(NB, dtype=torch.uint8, device="cuda")
buf.random_(0, 256)
scratch = torch.zeros(8, dtype=torch.int64, device="cuda")
sp = torch.cuda.current_stream().cuda_stream
names = {0: "gridstride 4x16B", 1: "one-shot wave 4KiB", 2: "one-shot wave 4KiB nt",
         3: "glds 4KiB", 4: "glds 4KiB aux=2", 5: "gridstride nt", 6: "glds 4KiB wpb4",
         7: "one-shot wpb4", 8: "glds aux=1", 9: "glds aux=3", 10: "glds 4-byte nt",
         11: "wpb1 contiguous", 12: "wpb1 contiguous nt", 13: "wpb1 rows", 14: "wpb1 rows nt"}
V = [int(x) for x in sys.argv[1:]] or sorted(names)
t = {v: [] for v in V}
for rnd in range(int(os.environ.get("AGN_PROBE_ROUNDS", "8"))):
    for v in V:
        b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        b.record()
        assert lib.agn_probe_variant(v, buf.data_ptr(), NB, scratch.data_ptr(), sp) == 0
        e.record()
        torch.cuda.synchronize()
        if rnd >= 2:
            t[v].append(b.elapsed_time(e))
for v in V:
    ms = float(np.median(t[v]))
    print(f"v{v} {names[v]:24s} {ms:.3f} ms  {NB / ms / 1e6:.0f} GB/s (best {NB / min(t[v]) / 1e6:.0f})",
          flush=True)
