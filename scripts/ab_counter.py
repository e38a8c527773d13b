"""A/B the counter_pn kernels (dense fast path vs general) on BASELINE cfg2 in
one process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from antidote_amd._lib import env_changed  # noqa: E402
from antidote_amd import _abi  # noqa: E402
from antidote_amd.engine import Engine  # noqa: E402

keys = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
eng = Engine(0)
cfg = _abi.AgnGenCfg(crdt_type=1, n_dcs=8, n_keys=keys, ops_per_key=64, n_elems=0,
                     seed=20250113, key_base=0, key_stride=1, warm=0)
dl, dr = eng.gen_dev(cfg)
VARS = {"key_w1": ("8", "1", None), "key_w2": ("8", "2", None), "key_w4": ("8", "4", None), "key_w8": ("8", "8", None), "v4g4": ("4", "4", None), "general": (None, None, "general")}
res = {v: eng.alloc_result(keys, 8, sparse=False) for v in VARS}
sp = torch.cuda.current_stream().cuda_stream
times = {v: [] for v in res}
for rnd in range(12):
    for v in res:
        var, minw, impl = VARS[v]
        for k, x in (("AGN_COUNTER_VARIANT", var), ("AGN_COUNTER_WPB", minw),
                     ("AGN_COUNTER_IMPL", impl)):
            if x is None:
                os.environ.pop(k, None)
                env_changed()
            else:
                os.environ[k] = x
                env_changed()
        b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        b.record()
        eng.materialize(dl, dr, res[v], stream=sp)
        e.record()
        torch.cuda.synchronize()
        if rnd >= 2:
            times[v].append(b.elapsed_time(e))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import probe_read_gbs  # noqa: E402
pr = probe_read_gbs(eng, dl, keys * 64 * 8 * 8, sp, torch)
print(f"probe read ceiling: {pr:.0f} GB/s")
os.environ.pop("AGN_COUNTER_IMPL", None)
env_changed()
os.environ.pop("AGN_COUNTER_VARIANT", None)
env_changed()
ref = eng.fetch_result(res["general"])
same = {}
for v in res:
    got = eng.fetch_result(res[v])
    same[v] = all(np.array_equal(getattr(got, f), getattr(ref, f)) for f in
                  ("value", "hole", "lastct", "count", "flags", "err_pos"))
byts = keys * 64 * 72 + keys * (8 + 16 * 8 + 32)
for v, t in times.items():
    ms = float(np.median(t))
    print(f"{v:8s} median {ms:.3f} ms  min {min(t):.3f}  {byts / ms / 1e6:.0f} GB/s  "
          f"{keys * 64 / ms / 1e6:.3e} ops/s  {byts / ms / 1e6 / pr:.3f} of probe")
print("outputs identical:", same)
