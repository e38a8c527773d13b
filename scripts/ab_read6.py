"""A/B of the fused cached read (agn_read_cached -> k_read6) at bulk size:
tools/libagn_prev.so's kernel (scripts/build_prev.sh) against the current
library with one / two requests per wave (AGN_READ6_NP), the XCD block order
(AGN_READ6_XCD) and the batched kernel sequence (AGN_READ_CACHED_SPLIT=1),
one process, interleaved rounds, the same device log / cache / result arrays
for all.  Two priming reads store every key's snapshot; each timed read is
then a cache hit with nothing to store (steady state), so every variant must
produce identical results.

  python scripts/ab_read6.py [config=2] [n_keys] [variants=prev,np1,np2,np2x,seq,name=lib.so]
"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from antidote_amd import _abi  # noqa: E402
from antidote_amd._lib import env_changed  # noqa: E402
from antidote_amd.engine import Engine  # noqa: E402
from bench import CONFIGS  # noqa: E402

c_id = int(sys.argv[1]) if len(sys.argv) > 1 else 2
cfg = CONFIGS[c_id]
K = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2] != "-" else cfg["n_keys"]
ONLY = sys.argv[3].split(",") if len(sys.argv) > 3 else ["prev", "np1", "np2", "np2x", "seq"]
D = cfg["n_dcs"]
assert cfg["crdt_type"] == 1 and D <= 8, "counter_pn, D <= 8"
VARS = {
    "prev": ("prev", {"AGN_READ_CACHED_SPLIT": "0"}),
    "np1": ("cur", {"AGN_READ_CACHED_SPLIT": "0", "AGN_READ6_NP": "1"}),
    "np2": ("cur", {"AGN_READ_CACHED_SPLIT": "0", "AGN_READ6_NP": "2"}),
    "np1x": ("cur", {"AGN_READ_CACHED_SPLIT": "0", "AGN_READ6_NP": "1", "AGN_READ6_XCD": "1"}),
    "np2x": ("cur", {"AGN_READ_CACHED_SPLIT": "0", "AGN_READ6_NP": "2", "AGN_READ6_XCD": "1"}),
    "seq": ("cur", {"AGN_READ_CACHED_SPLIT": "1"}),
    # runs of g blocks per XCD (block_order)
    **{f"np1c{g}": ("cur", {"AGN_READ_CACHED_SPLIT": "0", "AGN_READ6_NP": "1",
                            "AGN_READ6_XCD": str(g)}) for g in (16, 64, 128, 256)},
    **{f"np2c{g}": ("cur", {"AGN_READ_CACHED_SPLIT": "0", "AGN_READ6_NP": "2",
                            "AGN_READ6_XCD": str(g)}) for g in (32, 64, 128)},
    "default": ("cur", {}),
}
# name=path entries of the variant list: another library's fused kernel
EXTRA = dict(x.split("=", 1) for x in ONLY if "=" in x)
ONLY = [x.split("=", 1)[0] for x in ONLY]
VARS.update({n: (n, {"AGN_READ_CACHED_SPLIT": "0"}) for n in EXTRA})
VARS = {k: v for k, v in VARS.items() if k in ONLY}
KNOBS = sorted({k for _, e in VARS.values() for k in e})

eng = Engine(0)
LIBS = {}
for name, path in ([("prev", "tools/libagn_prev.so")] if "prev" in VARS else []) + list(EXTRA.items()):
    lib = C.CDLL(os.path.join(ROOT, path), mode=os.RTLD_LOCAL)
    _abi.bind(lib, {k: v for k, v in _abi.PROTOTYPES.items() if hasattr(lib, k)})
    ctx = C.c_void_p()
    assert lib.agn_open(0, C.byref(ctx)) == 0
    LIBS[name] = (lib, ctx)
sp = torch.cuda.current_stream().cuda_stream
g = _abi.AgnGenCfg(crdt_type=1, n_dcs=D, n_keys=K, ops_per_key=cfg["ops_per_key"],
                   n_elems=0, seed=cfg["seed"], key_base=0, key_stride=1, warm=0)
dl, dr = eng.gen_dev(g)
S = _abi.SNAPSHOT_THRESHOLD
bufs = {"n": eng.empty(4 * K), "clock": eng.empty(8 * K * S * D), "last_op": eng.empty(8 * K * S),
        "value": eng.empty(8 * K * S), "status": eng.empty(K), "prune": eng.empty(K),
        "thr": eng.empty(8 * K * D)}
eng.lib.agn_memset_d(eng.ctx, bufs["n"].ptr, 0, 4 * K, sp)
cache = _abi.AgnSsCache()
cache.n_dcs, cache.slots, cache.n_keys = D, S, K
cache.n, cache.clock, cache.last_op, cache.value = (bufs[x].ptr for x in ("n", "clock", "last_op", "value"))
res = eng.alloc_result(K, D, sparse=False)
dkeys = eng.upload(np.arange(K, dtype=np.uint64))


def set_env(env):
    for k in KNOBS:
        os.environ.pop(k, None)
    os.environ.update(env)
    env_changed()
    for lib, _ in LIBS.values():
        if hasattr(lib, "agn_env_reload"):
            lib.agn_env_reload()


def run(lib):
    if lib == "cur":
        eng.read_cached(cache, dl, K, dkeys.ptr, dr.R, dr.txid, None, res, bufs["status"].ptr,
                        bufs["prune"].ptr, bufs["thr"].ptr, sp)
    else:
        L, ctx = LIBS[lib]
        rc = L.agn_read_cached(ctx, C.byref(cache), C.byref(dl), K, dkeys.ptr, dr.R, dr.txid,
                               None, C.byref(res.struct), bufs["status"].ptr, bufs["prune"].ptr,
                               bufs["thr"].ptr, sp)
        assert rc == 0


def snapshot():
    torch.cuda.synchronize()
    r = eng.fetch_result(res)
    out = {f: getattr(r, f) for f in ("value", "hole", "lastct", "count", "flags", "err_pos")}
    out["status"] = eng.download(bufs["status"], np.uint8, (K,))
    out["prune"] = eng.download(bufs["prune"], np.uint8, (K,))
    out["n"] = eng.download(bufs["n"], np.uint32, (K,))
    return out


set_env({"AGN_READ_CACHED_SPLIT": "1"})
run("cur")  # priming: absent keys -> empty snapshot -> cold read -> store
run("cur")
names = list(VARS)
times = {v: [] for v in names}
outs = {}
for rnd in range(12):
    order = names[rnd % len(names):] + names[:rnd % len(names)]
    for v in order:
        lib, env = VARS[v]
        set_env(env)
        b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        b.record()
        run(lib)
        e.record()
        torch.cuda.synchronize()
        if rnd >= 2:
            times[v].append(b.elapsed_time(e))
        if rnd == 0:
            outs[v] = snapshot()
set_env({})
ref = outs[names[0]]
summary = {"config": c_id, "n_keys": K, "n_dcs": D,
           "hit_frac": float((ref["status"] == _abi.SS_HIT).mean()), "ms_median": {}, "ms_min": {},
           "identical": {}}
for v, t in times.items():
    summary["ms_median"][v] = float(np.median(t))
    summary["ms_min"][v] = float(min(t))
    summary["identical"][v] = all(np.array_equal(outs[v][f], ref[f]) for f in ref)
print(json.dumps(summary), flush=True)
