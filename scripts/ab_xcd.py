"""A/B the XCD-aware block order (AGN_XCD_REMAP=0|1) on the cfg2/cfg3/cfg4
materialize kernels, interleaved in one process (box-to-box HBM variance is
+-4 %, so variants are only compared inside one run)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from antidote_amd._lib import env_changed  # noqa: E402
from antidote_amd import _abi  # noqa: E402
from antidote_amd.engine import Engine  # noqa: E402
from bench import CONFIGS, algorithmic_bytes, probe_read_gbs  # noqa: E402

FIELDS = ("value", "hole", "lastct", "count", "flags", "err_pos")
eng = Engine(0)
sp = torch.cuda.current_stream().cuda_stream
cfgs = [int(c) for c in (sys.argv[1:] or ["2", "3", "4"])]
for c in cfgs:
    cfg = CONFIGS[c]
    K = cfg["n_keys"]
    g = _abi.AgnGenCfg(crdt_type=cfg["crdt_type"], n_dcs=cfg["n_dcs"], n_keys=K,
                       ops_per_key=cfg["ops_per_key"], n_elems=cfg["n_elems"], seed=cfg["seed"],
                       key_base=0, key_stride=1, warm=0)
    dl, dr = eng.gen_dev(g)
    cap = None
    if cfg["crdt_type"] != 1:
        cap = np.arange(K + 1, dtype=np.uint64) * np.uint64(cfg["ops_per_key"])
    VAR = ["0", "1"]
    res = {x: eng.alloc_result(K, cfg["n_dcs"], sparse=False, cap_off=cap) for x in VAR}
    n_rem = 0
    if cfg["crdt_type"] != 1:
        E = K * cfg["ops_per_key"]
        n_rem = int(eng.download(type("B", (), {"ptr": dl.rem_off})(), np.uint32, (E + 1,))[-1])
    times = {x: [] for x in VAR}
    for rnd in range(14):
        for x in VAR:
            os.environ["AGN_XCD_REMAP"] = x
            env_changed()
            b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            b.record()
            eng.materialize(dl, dr, res[x], stream=sp)
            e.record()
            torch.cuda.synchronize()
            if rnd >= 2:
                times[x].append(b.elapsed_time(e))
    outs = {x: eng.fetch_result(res[x]) for x in VAR}
    fields = FIELDS if cfg["crdt_type"] == 1 else FIELDS[1:] + ("out_n", "out_tag", "out_tok")
    n_live = 0 if cfg["crdt_type"] == 1 else int(outs["0"].out_n.astype(np.int64).sum())
    byts = algorithmic_bytes(cfg, K, n_rem, n_live)
    pr = probe_read_gbs(eng, dl, K * cfg["ops_per_key"] * cfg["n_dcs"] * 8, sp, torch)
    for x, t in times.items():
        ms = float(np.median(t))
        same = all(np.array_equal(getattr(outs[x], f), getattr(outs["0"], f)) for f in fields)
        print(f"cfg{c} xcd={x} median {ms:.3f} ms min {min(t):.3f}  {byts / ms / 1e6:.0f} GB/s  "
              f"{byts / ms / 1e6 / 8000:.3f} of 8 TB/s  {byts / ms / 1e6 / pr:.3f} of probe "
              f"({pr:.0f})  same={same}", flush=True)
    eng.free_gen(dl, dr)
    for r in res.values():
        for bb in r.bufs.values():
            bb.free()
os.environ.pop("AGN_XCD_REMAP", None)
env_changed()
