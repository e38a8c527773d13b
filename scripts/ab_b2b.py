"""Back-to-back (bench-style) vs synchronised (A/B-style) launches of the
cfg2 counter kernel, for the VGPR and LDS-DMA row paths, in one process."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from antidote_amd._lib import env_changed  # noqa: E402
from antidote_amd import _abi  # noqa: E402
from antidote_amd.engine import Engine  # noqa: E402
from bench import CONFIGS, probe_read_gbs  # noqa: E402

cfg = CONFIGS[2]
K = cfg["n_keys"]
eng = Engine(0)
sp = torch.cuda.current_stream().cuda_stream
g = _abi.AgnGenCfg(crdt_type=1, n_dcs=8, n_keys=K, ops_per_key=64, n_elems=0, seed=cfg["seed"],
                   key_base=0, key_stride=1, warm=0)
dl, dr = eng.gen_dev(g)
res = eng.alloc_result(K, 8, sparse=False)
byts = K * 64 * 72 + K * 168
for rnd in range(3):
    for glds in ("0", "1"):
        os.environ["AGN_COUNTER_GLDS"] = glds
        env_changed()
        for _ in range(2):
            eng.materialize(dl, dr, res, stream=sp)
        torch.cuda.synchronize()
        # back-to-back
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(20)]
        for b, e in ev:
            b.record()
            eng.materialize(dl, dr, res, stream=sp)
            e.record()
        torch.cuda.synchronize()
        t_b2b = [b.elapsed_time(e) for b, e in ev]
        # synchronised
        t_sync = []
        for _ in range(20):
            b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            b.record()
            eng.materialize(dl, dr, res, stream=sp)
            e.record()
            torch.cuda.synchronize()
            t_sync.append(b.elapsed_time(e))
        print(f"round {rnd} glds={glds}: b2b mean {np.mean(t_b2b):.3f} ms (first {t_b2b[0]:.3f}, "
              f"last {t_b2b[-1]:.3f})  sync median {np.median(t_sync):.3f} ms  "
              f"-> {byts / np.mean(t_b2b) / 1e6:.0f} / {byts / np.median(t_sync) / 1e6:.0f} GB/s",
              flush=True)
print(f"probe {probe_read_gbs(eng, dl, K * 64 * 64, sp, torch):.0f} GB/s")
