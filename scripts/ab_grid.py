"""A/B the group-stream counter kernel's grid size (one process, interleaved)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from antidote_amd._lib import env_changed  # noqa: E402
from antidote_amd import _abi  # noqa: E402
from antidote_amd.engine import Engine  # noqa: E402

keys = 10_000_000
eng = Engine(0)
cfg = _abi.AgnGenCfg(crdt_type=1, n_dcs=8, n_keys=keys, ops_per_key=64, n_elems=0,
                     seed=20250113, key_base=0, key_stride=1, warm=0)
dl, dr = eng.gen_dev(cfg)
var = sys.argv[1] if len(sys.argv) > 1 else "4"
GRIDS = ["196608", "625000", "1250000", "2500000"]
res = eng.alloc_result(keys, 8, sparse=False)
sp = torch.cuda.current_stream().cuda_stream
os.environ["AGN_COUNTER_VARIANT"] = var
env_changed()
times = {g: [] for g in GRIDS}
for rnd in range(8):
    for g in GRIDS:
        os.environ["AGN_GROUP_BLOCKS"] = g
        env_changed()
        if g == "0":
            os.environ.pop("AGN_GROUP_BLOCKS")
            env_changed()
        b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        b.record()
        eng.materialize(dl, dr, res, stream=sp)
        e.record()
        torch.cuda.synchronize()
        if rnd >= 2:
            times[g].append(b.elapsed_time(e))
byts = keys * 64 * 72 + keys * (8 + 16 * 8 + 32)
for g, t in times.items():
    ms = float(np.median(t))
    print(f"var {var} grid {g:>6s}  median {ms:.3f} ms  {byts / ms / 1e6:.0f} GB/s")
