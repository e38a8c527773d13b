"""Generic env-knob A/B of the materialize kernels, interleaved in one process.

  python scripts/ab_env.py --cfg 2 --cfg 4 --var base: --var glds:AGN_COUNTER_GLDS=1,AGN_X=0

Each --var is NAME:K=V[,K=V...] (empty = defaults).  Outputs are compared
with the first variant's (bit-exact), bytes/s against 8 TB/s and the probe."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from antidote_amd._lib import env_changed  # noqa: E402
from antidote_amd import _abi  # noqa: E402
from antidote_amd.engine import Engine  # noqa: E402
from bench import CONFIGS, algorithmic_bytes, probe_read_gbs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cfg", type=int, action="append", default=[])
ap.add_argument("--var", action="append", default=[])
ap.add_argument("--rounds", type=int, default=12)
ap.add_argument("--keys", type=int, default=0)
ap.add_argument("--warm", type=int, default=0)
a = ap.parse_args()
VARS = {}
for v in a.var:
    name, _, kv = v.partition(":")
    VARS[name] = dict(x.split("=", 1) for x in kv.split(",") if x)
KNOBS = sorted({k for d in VARS.values() for k in d})
FIELDS = ("value", "hole", "lastct", "count", "flags", "err_pos")
eng = Engine(0)
sp = torch.cuda.current_stream().cuda_stream
for c in a.cfg or [2]:
    cfg = CONFIGS[c]
    K = a.keys or cfg["n_keys"]
    g = _abi.AgnGenCfg(crdt_type=cfg["crdt_type"], n_dcs=cfg["n_dcs"], n_keys=K,
                       ops_per_key=cfg["ops_per_key"], n_elems=cfg["n_elems"], seed=cfg["seed"],
                       key_base=0, key_stride=1, warm=a.warm)
    dl, dr = eng.gen_dev(g)
    cap = None
    if cfg["crdt_type"] != 1:
        cap = np.arange(K + 1, dtype=np.uint64) * np.uint64(cfg["ops_per_key"])
    # one shared result buffer (per-variant buffers biased the first variant's
    # timing by 1-3 %), variant order rotated every round
    res = eng.alloc_result(K, cfg["n_dcs"], sparse=False, cap_off=cap)
    n_rem = 0
    if cfg["crdt_type"] != 1:
        E = K * cfg["ops_per_key"]
        n_rem = int(eng.download(type("B", (), {"ptr": dl.rem_off})(), np.uint32, (E + 1,))[-1])
    names = list(VARS)
    times = {x: [] for x in VARS}

    def setenv(env):
        for k in KNOBS:
            if k in env:
                os.environ[k] = env[k]
                env_changed()
            else:
                os.environ.pop(k, None)
                env_changed()

    for rnd in range(a.rounds):
        order = names[rnd % len(names):] + names[:rnd % len(names)]
        for x in order:
            setenv(VARS[x])
            b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            b.record()
            eng.materialize(dl, dr, res, stream=sp)
            e.record()
            torch.cuda.synchronize()
            if rnd >= 2:
                times[x].append(b.elapsed_time(e))
    outs = {}
    for x in names:
        setenv(VARS[x])
        eng.materialize(dl, dr, res, stream=sp)
        torch.cuda.synchronize()
        outs[x] = eng.fetch_result(res)
    for k in KNOBS:
        os.environ.pop(k, None)
        env_changed()
    first = next(iter(VARS))
    fields = FIELDS if cfg["crdt_type"] == 1 else FIELDS[1:] + ("out_n", "out_tag", "out_tok")
    n_live = 0 if cfg["crdt_type"] == 1 else int(outs[first].out_n.astype(np.int64).sum())
    byts = algorithmic_bytes(cfg, K, n_rem, n_live)
    pr = probe_read_gbs(eng, dl, K * cfg["ops_per_key"] * cfg["n_dcs"] * 8, sp, torch)
    for x, t in times.items():
        ms = float(np.median(t))
        same = all(np.array_equal(getattr(outs[x], f), getattr(outs[first], f)) for f in fields)
        print(f"cfg{c} {x:10s} median {ms:.3f} ms min {min(t):.3f}  {byts / ms / 1e6:.0f} GB/s  "
              f"{byts / ms / 1e6 / 8000:.3f} of 8 TB/s  {byts / ms / 1e6 / pr:.3f} of probe "
              f"({pr:.0f})  same={same}", flush=True)
    eng.free_gen(dl, dr)
    for bb in res.bufs.values():
        bb.free()
