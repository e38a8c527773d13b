"""A/B the tag-resolution kernel's grid (cfg3 / cfg4 shapes, one process)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from antidote_amd import _abi  # noqa: E402
from antidote_amd.engine import Engine  # noqa: E402
from bench import CONFIGS, algorithmic_bytes  # noqa: E402

eng = Engine(0)
sp = torch.cuda.current_stream().cuda_stream
for c in (3, 4):
    cfg = CONFIGS[c]
    K = cfg["n_keys"]
    g = _abi.AgnGenCfg(crdt_type=cfg["crdt_type"], n_dcs=cfg["n_dcs"], n_keys=K,
                       ops_per_key=cfg["ops_per_key"], n_elems=cfg["n_elems"], seed=cfg["seed"],
                       key_base=0, key_stride=1, warm=0)
    dl, dr = eng.gen_dev(g)
    cap = np.arange(K + 1, dtype=np.uint64) * np.uint64(cfg["ops_per_key"])
    res = eng.alloc_result(K, cfg["n_dcs"], sparse=False, cap_off=cap)
    E = K * cfg["ops_per_key"]
    n_rem = int(eng.download(type("B", (), {"ptr": dl.rem_off})(), np.uint32, (E + 1,))[-1])
    GR = ["0"]
    times = {x: [] for x in GR}
    outs = {}
    for rnd in range(6):
        for x in GR:
            if x == "0":
                os.environ.pop("AGN_TAGS_GRID", None)
            else:
                os.environ["AGN_TAGS_GRID"] = x
            b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            b.record()
            eng.materialize(dl, dr, res, stream=sp)
            e.record()
            torch.cuda.synchronize()
            if rnd >= 1:
                times[x].append(b.elapsed_time(e))
            if rnd == 5:
                outs[x] = eng.fetch_result(res)
    n_live = int(outs["0"].out_n.astype(np.int64).sum())
    byts = algorithmic_bytes(cfg, K, n_rem, n_live)
    ref = outs["0"]
    for x, t in times.items():
        ms = float(np.median(t))
        same = all(np.array_equal(getattr(outs[x], f), getattr(ref, f)) for f in
                   ("hole", "lastct", "count", "flags", "out_n", "out_tag", "out_tok"))
        print(f"cfg{c} grid {x:>6s} median {ms:.3f} ms  {byts / ms / 1e6:.0f} GB/s  same={same}")
    eng.free_gen(dl, dr)
    for bb in res.bufs.values():
        bb.free()
os.environ.pop("AGN_TAGS_GRID", None)
