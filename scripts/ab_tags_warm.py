"""A/B of the warm set_aw / register_mv materialize (k_tags from the cached
states, bench.py --warm's cfg3 / cfg4 sub-line) between the current library
and other builds (name=lib.so, e.g. tools/libagn_prev.so from
scripts/build_prev.sh), one process, interleaved rounds with rotating order.
The cache is primed as bench.py's warm_bench_tags does (two cold reads +
stores); each timed step is then a lookup (current library) and the warm
materialize of the variant, with no store, so every variant reads the same
cached states and must produce identical results.

  python scripts/ab_tags_warm.py [config=3] [name=lib.so ...]
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
from antidote_amd.engine import Engine  # noqa: E402
from bench import CONFIGS  # noqa: E402

c_id = int(sys.argv[1]) if len(sys.argv) > 1 else 3
cfg = CONFIGS[c_id]
assert cfg["crdt_type"] != 1, "set_aw / register_mv configs"
K, D, N = cfg["n_keys"], cfg["n_dcs"], cfg["ops_per_key"]
eng = Engine(0)
LIBS = {}
for a in (sys.argv[2:] or ["prev=tools/libagn_prev.so"]):
    name, path = a.split("=", 1)
    lib = C.CDLL(os.path.join(ROOT, path), mode=os.RTLD_LOCAL)
    _abi.bind(lib, {k: v for k, v in _abi.PROTOTYPES.items() if hasattr(lib, k)})
    ctx = C.c_void_p()
    assert lib.agn_open(0, C.byref(ctx)) == 0
    LIBS[name] = (lib, ctx)
sp = torch.cuda.current_stream().cuda_stream
g = _abi.AgnGenCfg(crdt_type=cfg["crdt_type"], n_dcs=D, n_keys=K, ops_per_key=N,
                   n_elems=cfg["n_elems"], seed=cfg["seed"], key_base=0, key_stride=1, warm=0)
dl, dr = eng.gen_dev(g)
S = _abi.SNAPSHOT_THRESHOLD
cap_off = np.arange(K + 1, dtype=np.uint64) * np.uint64(N)
arena_cap = 2 * K * N
bufs = {"n": eng.empty(4 * K), "clock": eng.empty(8 * K * S * D), "last_op": eng.empty(8 * K * S),
        "value": eng.empty(8 * K * S), "sct": eng.empty(8 * K * D), "ign": eng.empty(K),
        "base": eng.empty(8 * K), "first": eng.empty(K), "status": eng.empty(K),
        "prune": eng.empty(K), "thr": eng.empty(8 * K * D), "ctl": eng.empty(32),
        "st_tag": eng.empty(4 * arena_cap), "st_tok": eng.empty(8 * arena_cap)}
eng.lib.agn_memset_d(eng.ctx, bufs["n"].ptr, 0, 4 * K, sp)
eng.lib.agn_memset_d(eng.ctx, bufs["ctl"].ptr, 0, 32, sp)
cache = _abi.AgnSsCache()
cache.n_dcs, cache.slots, cache.n_keys = D, S, K
cache.n, cache.clock, cache.last_op, cache.value = (bufs[x].ptr for x in ("n", "clock", "last_op", "value"))
cache.state_tag, cache.state_tok, cache.state_cap, cache.state_ctl = (
    bufs["st_tag"].ptr, bufs["st_tok"].ptr, arena_cap, bufs["ctl"].ptr)
req = _abi.AgnRead()
C.memmove(C.addressof(req), C.addressof(dr), C.sizeof(_abi.AgnRead))
req.sct, req.sct_ignore, req.base_value = bufs["sct"].ptr, bufs["ign"].ptr, bufs["base"].ptr
req.base_off, req.base_tag, req.base_tok = None, bufs["st_tag"].ptr, bufs["st_tok"].ptr
res = eng.alloc_result(K, D, sparse=False, cap_off=cap_off)


def lookup():
    eng.ss_lookup(cache, K, None, dr.R, None, bufs["sct"].ptr, None, bufs["ign"].ptr,
                  bufs["base"].ptr, bufs["first"].ptr, bufs["status"].ptr, sp)


def store():
    eng.ss_store(cache, dl, K, None, bufs["first"].ptr, bufs["status"].ptr, None, res, None,
                 bufs["prune"].ptr, bufs["thr"].ptr, None, sp)


def run(v):
    if v == "cur":
        eng.materialize(dl, req, res, sp)
    else:
        L, ctx = LIBS[v]
        assert L.agn_materialize(ctx, C.byref(dl), C.byref(req), C.byref(res.struct), sp) == 0


for _ in range(2):  # priming: absent keys -> empty snapshot -> cold read -> store
    lookup()
    eng.materialize(dl, req, res, sp)
    store()
names = ["cur"] + list(LIBS)
times = {v: [] for v in names}
outs = {}
fields = ["hole", "lastct", "count", "flags", "err_pos", "out_n", "out_tag", "out_tok"]
for rnd in range(12):
    order = names[rnd % len(names):] + names[:rnd % len(names)]
    for v in order:
        lookup()
        b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        b.record()
        run(v)
        e.record()
        torch.cuda.synchronize()
        if rnd >= 2:
            times[v].append(b.elapsed_time(e))
        if rnd == 0:
            r = eng.fetch_result(res)
            outs[v] = {f: getattr(r, f) for f in fields}
hits = eng.download(bufs["status"], np.uint8, (K,))
ref = outs["cur"]
summary = {"config": c_id, "n_keys": K, "hit_frac": float((hits == _abi.SS_HIT).mean()),
           "ms_median": {}, "ms_min": {}, "identical": {}}
for v, t in times.items():
    summary["ms_median"][v] = float(np.median(t))
    summary["ms_min"][v] = float(min(t))
    summary["identical"][v] = all(np.array_equal(outs[v][f], ref[f]) for f in ref)
print(json.dumps(summary), flush=True)
