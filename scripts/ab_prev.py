"""A/B the current library against tools/libagn_prev.so (an earlier commit,
scripts/build_prev.sh) on BASELINE cfg2, one process, interleaved rounds with
rotating order; both libraries share the process's HIP runtime, so the same
device log / request / result buffers feed both.  WARM=1: warm requests
(snapshot-carrying, the k_counter_quad2 path for counters)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from antidote_amd._lib import env_changed  # noqa: E402
from antidote_amd import _abi  # noqa: E402
from antidote_amd.engine import Engine  # noqa: E402
from bench import CONFIGS, algorithmic_bytes, probe_read_gbs  # noqa: E402

c = int(sys.argv[1]) if len(sys.argv) > 1 else 2
cfg = CONFIGS[c]
K = cfg["n_keys"]
eng = Engine(0)
# extra libraries: name=path arguments (default: prev=tools/libagn_prev.so)
LIBS = {}
ENV_VARS = {}
for a in (sys.argv[2:] or ["prev=tools/libagn_prev.so"]):
    name, path = a.split("=", 1)
    if path.startswith("env:"):  # name=env:KEY=VAL: the current library with an env knob
        k, v = path[4:].split("=", 1)
        ENV_VARS[name] = {k: v}
        continue
    lib = C.CDLL(os.path.join(ROOT, path), mode=os.RTLD_LOCAL)
    _abi.bind(lib, {k: v for k, v in _abi.PROTOTYPES.items() if hasattr(lib, k)})
    ctx = C.c_void_p()
    assert lib.agn_open(0, C.byref(ctx)) == 0
    LIBS[name] = (lib, ctx)
sp = torch.cuda.current_stream().cuda_stream
g = _abi.AgnGenCfg(crdt_type=cfg["crdt_type"], n_dcs=cfg["n_dcs"], n_keys=K,
                   ops_per_key=cfg["ops_per_key"], n_elems=cfg["n_elems"], seed=cfg["seed"],
                   key_base=0, key_stride=1, warm=int(os.environ.get("WARM", "0")))
dl, dr = eng.gen_dev(g)
cap = None
if cfg["crdt_type"] != 1:
    cap = np.arange(K + 1, dtype=np.uint64) * np.uint64(cfg["ops_per_key"])
res = eng.alloc_result(K, cfg["n_dcs"], sparse=False, cap_off=cap)
rec = eng.empty(K * 128) if any(n.startswith("rec") for n in LIBS) else None
ENVS = {"AGN_COUNTER_ID0", "AGN_COUNTER_GLDS"} | {k for e in ENV_VARS.values() for k in e}
VARS = {"cur": ("cur", {})}
VARS.update({n: (n, {}) for n in LIBS})
VARS.update({n: ("cur", e) for n, e in ENV_VARS.items()})


def run(lib):
    if lib == "cur":
        eng.materialize(dl, dr, res, stream=sp)
    else:
        L, ctx = LIBS[lib]
        saved = res.struct.err_pos
        if lib.startswith("rec"):  # diagnostic record layout: 128 B per key into `rec`
            res.struct.err_pos = rec.ptr
        rc = L.agn_materialize(ctx, C.byref(dl), C.byref(dr), C.byref(res.struct), sp)
        res.struct.err_pos = saved
        assert rc == 0


names = list(VARS)
times = {v: [] for v in names}
outs = {}
for rnd in range(14):
    order = names[rnd % len(names):] + names[:rnd % len(names)]
    for v in order:
        lib, env = VARS[v]
        for k in ENVS:
            os.environ.pop(k, None)
            env_changed()
        os.environ.update(env)
        env_changed()
        b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        b.record()
        run(lib)
        e.record()
        torch.cuda.synchronize()
        if rnd >= 2:
            times[v].append(b.elapsed_time(e))
        if rnd == 0:
            outs[v] = eng.fetch_result(res)
for k in ENVS:
    os.environ.pop(k, None)
    env_changed()
pr = probe_read_gbs(eng, dl, K * cfg["ops_per_key"] * cfg["n_dcs"] * 8, sp, torch)
n_rem = n_live = 0
if cfg["crdt_type"] != 1:
    E = K * cfg["ops_per_key"]
    n_rem = int(eng.download(type("B", (), {"ptr": dl.rem_off})(), np.uint32, (E + 1,))[-1])
    n_live = int(eng.download(res.bufs["out_n"], np.uint32, (K,)).astype(np.int64).sum())
byts = algorithmic_bytes(cfg, K, n_rem, n_live)
print(f"cfg{c} probe read ceiling: {pr:.0f} GB/s")
ref = outs["cur"]
fields = ["value", "hole", "lastct", "count", "flags", "err_pos"]
if cfg["crdt_type"] != 1:
    fields = ["hole", "lastct", "count", "flags", "err_pos", "out_n"]
for v, t in times.items():
    ms = float(np.median(t))
    same = all(np.array_equal(getattr(outs[v], f), getattr(ref, f)) for f in fields)
    print(f"cfg{c} {v:7s} median {ms:.3f} ms  min {min(t):.3f}  {byts / ms / 1e6:.0f} GB/s  "
          f"{byts / ms / 1e6 / 8000:.3f} of 8 TB/s  {byts / ms / 1e6 / pr:.3f} of probe  "
          f"identical={same}")
