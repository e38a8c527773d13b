"""A/B the counter dense kernel with and without agn_log.key_id0 (NewLastOp
from the consecutive-id index vs a dependent op_id load) on BASELINE cfg2, one
process, interleaved rounds with rotating order."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from antidote_amd._lib import env_changed  # noqa: E402
from antidote_amd import _abi  # noqa: E402
from antidote_amd.engine import Engine  # noqa: E402
from bench import probe_read_gbs  # noqa: E402

keys = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
eng = Engine(0)
cfg = _abi.AgnGenCfg(crdt_type=1, n_dcs=8, n_keys=keys, ops_per_key=64, n_elems=0,
                     seed=20250113, key_base=0, key_stride=1, warm=0)
dl, dr = eng.gen_dev(cfg)
VARS = {"id0": {}, "load": {"AGN_COUNTER_ID0": "0"},
        "pair": {"AGN_COUNTER_KPW": "2"}, "pair_ld": {"AGN_COUNTER_KPW": "2", "AGN_COUNTER_ID0": "0"}}
res = eng.alloc_result(keys, 8, sparse=False)
sp = torch.cuda.current_stream().cuda_stream
times = {v: [] for v in VARS}
outs = {}
names = list(VARS)
for rnd in range(14):
    order = names[rnd % len(names):] + names[:rnd % len(names)]
    for v in order:
        for k in ("AGN_COUNTER_ID0", "AGN_COUNTER_GLDS", "AGN_COUNTER_KPW"):
            os.environ.pop(k, None)
            env_changed()
        os.environ.update(VARS[v])
        env_changed()
        b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        b.record()
        eng.materialize(dl, dr, res, stream=sp)
        e.record()
        torch.cuda.synchronize()
        if rnd >= 2:
            times[v].append(b.elapsed_time(e))
        if rnd == 0:
            outs[v] = eng.fetch_result(res)
pr = probe_read_gbs(eng, dl, keys * 64 * 8 * 8, sp, torch)
print(f"probe read ceiling: {pr:.0f} GB/s")
ref = outs["load"]
byts = keys * 64 * 72 + keys * (8 + 16 * 8 + 32)
for v, t in times.items():
    ms = float(np.median(t))
    same = all(np.array_equal(getattr(outs[v], f), getattr(ref, f)) for f in
               ("value", "hole", "lastct", "count", "flags", "err_pos"))
    print(f"{v:6s} median {ms:.3f} ms  min {min(t):.3f}  {byts / ms / 1e6:.0f} GB/s  "
          f"{byts / ms / 1e6 / 8000:.3f} of 8 TB/s  {byts / ms / 1e6 / pr:.3f} of probe  "
          f"identical={same}")
