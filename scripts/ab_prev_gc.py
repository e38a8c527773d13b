"""A/B of the one-pass segmented GC (agn_prune_ops with out.key_len, the
k_prune_inplace kernel bench.py --gc times) between the current library and
tools/libagn_prev.so (scripts/build_prev.sh), one process, interleaved rounds,
the same device log / thresholds / output arrays for both; the outputs must
be identical.

  python scripts/ab_prev_gc.py [config=3] [name=path ...]

name=path: more libraries (default prev=tools/libagn_prev.so), e.g. the
diagnostic builds of scripts/build_diag_gc.sh (their outputs differ by
design: `identical` is reported, not asserted).
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from antidote_amd import _abi  # noqa: E402
from antidote_amd.engine import DeviceArrays, Engine  # noqa: E402
from bench import CONFIGS, HBM_PEAK_GBS  # noqa: E402

c = int(sys.argv[1]) if len(sys.argv) > 1 else 3
cfg = CONFIGS[c]
K, D, N = cfg["n_keys"], cfg["n_dcs"], cfg["ops_per_key"]
E = K * N
tags = cfg["crdt_type"] != 1
eng = Engine(0)
from antidote_amd._lib import env_changed  # noqa: E402

LIBS, ENVS = {}, {}
for a in (sys.argv[2:] or ["prev=tools/libagn_prev.so"]):
    name, path = a.split("=", 1)
    if path.startswith("env:"):  # name=env:K=V[,K=V]: the current library with knobs
        ENVS[name] = dict(kv.split("=", 1) for kv in path[4:].split(","))
        continue
    lib = C.CDLL(os.path.join(ROOT, path), mode=os.RTLD_LOCAL)
    _abi.bind(lib, {k: v for k, v in _abi.PROTOTYPES.items() if hasattr(lib, k)})
    ctx = C.c_void_p()
    assert lib.agn_open(0, C.byref(ctx)) == 0
    LIBS[name] = (lib, ctx)
sp = torch.cuda.current_stream().cuda_stream
g = _abi.AgnGenCfg(crdt_type=cfg["crdt_type"], n_dcs=D, n_keys=K, ops_per_key=N,
                   n_elems=cfg["n_elems"], seed=cfg["seed"], key_base=0, key_stride=1, warm=0)
dl, dr = eng.gen_dev(g)
s = _abi.AgnLog()
s.crdt_type, s.n_dcs, s.n_keys, s.n_entries = cfg["crdt_type"], D, K, E
out = DeviceArrays(s)
spec = {"key_off": 8 * (K + 1), "oc": 8 * E * D, "op_id": 4 * E, "txid": 8 * E}
if tags:
    n_rem = int(eng.download(type("B", (), {"ptr": dl.rem_off})(), np.uint32, (E + 1,))[-1])
    spec.update({"tag": 4 * E, "add_tok": 8 * E, "rem_off": 4 * (E + 1),
                 "rem_tok": 8 * max(n_rem, 1)})
else:
    spec["eff"] = 8 * E
for name, nb in spec.items():
    b = eng.empty(nb)
    out.bufs[name] = b
    setattr(s, name, b.ptr)
key_len = eng.empty(8 * K)
s.key_len = key_len.ptr
tot = eng.empty(16)


KNOBS = {k for e in ENVS.values() for k in e}


def run(lib):
    for k in KNOBS:
        os.environ.pop(k, None)
    if lib in ENVS:
        os.environ.update(ENVS[lib])
    env_changed()
    if lib == "cur" or lib in ENVS:
        rc = eng.lib.agn_prune_ops(eng.ctx, C.byref(dl), None, dr.R, None, C.byref(s), None,
                                   tot.ptr, sp)
    else:
        lib, ctx = LIBS[lib]
        rc = lib.agn_prune_ops(ctx, C.byref(dl), None, dr.R, None, C.byref(s), None, tot.ptr, sp)
    assert rc == 0


def snapshot():
    torch.cuda.synchronize()
    return {n: eng.download(b, np.uint8, (spec[n],)) for n, b in out.bufs.items()} | \
        {"key_len": eng.download(key_len, np.uint64, (K,))}


names = ["cur"] + list(LIBS) + list(ENVS)
times = {v: [] for v in names}
outs = {}
for rnd in range(10):
    for v in names[rnd % len(names):] + names[:rnd % len(names)]:
        b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        b.record()
        run(v)
        e.record()
        torch.cuda.synchronize()
        if rnd >= 2:
            times[v].append(b.elapsed_time(e))
        if rnd == 0:
            outs[v] = snapshot()
kept, kept_rem = (int(x) for x in eng.download(tot, np.uint64, (2,)))
per_f = 4 + 8 + (16 if tags else 8)
alg = E * 8 * D + kept * per_f * 2 + kept * 8 * D + 16 * kept_rem + K * (8 + 8 * D + 16)
for v, t in times.items():
    ms = float(np.median(t))
    same = all(np.array_equal(outs["cur"][n], outs[v][n]) for n in outs["cur"])
    print(f"cfg{c} gc {v:5s} median {ms:.3f} ms  min {min(t):.3f}  "
          f"{alg / ms / 1e6:.0f} GB/s  {alg / ms / 1e6 / HBM_PEAK_GBS:.3f} of 8 TB/s  identical={same}",
          flush=True)
