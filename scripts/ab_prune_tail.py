"""A/B of the engine-owned log's GC kernel (agn_oplog_prune -> k_prune_tail)
on the prefix-drop workload of scripts/bench_oplog_prune.py (K keys x N ops,
D = 8, threshold = the clock of a random position), variants alternated in
one process on fresh logs (HBM rates move several % between processes):
  AGN_PRUNE_WPB = 1 | 4 (waves per block), AGN_PRUNE_TAIL_MINW = 1 | 8 (the
  compiler's register allocation, 7 waves per SIMD, or the budget of 8: the
  default since round 3), AGN_PRUNE_TAIL_KPW = 2 | 4 (keys per wave, every
  key's metadata and newest chunk in flight before the first is walked).
Times the prune call's GPU span (events on the log's stream: the kernel plus
the records' copy) and checks that both variants leave identical logs.

  python scripts/ab_prune_tail.py [K] [N] [rounds]
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from antidote_amd._lib import env_changed  # noqa: E402
from antidote_amd import _abi  # noqa: E402
from antidote_amd.engine import Engine, OpLog  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    D = 8
    rng = np.random.default_rng(7)
    keys = np.repeat(np.arange(K, dtype=np.uint64), N)
    pos = np.tile(np.arange(N, dtype=np.uint64), K)
    oc = (np.uint64(1_700_000_000_000_000) + pos[:, None] * np.uint64(1000)
          + rng.integers(0, 500, (K * N, D), dtype=np.uint64))
    eff = rng.integers(-1000, 1001, K * N, dtype=np.int64)
    txid = np.zeros(K * N, np.uint64)
    cut = rng.integers(0, N, K)
    thr = oc.reshape(K, N, D)[np.arange(K), cut].copy()
    prune = np.ones(K, np.uint8)
    import torch
    torch.cuda.init()
    eng = Engine(0)
    bp, bt = eng.upload(prune), eng.upload(thr)
    fl = eng.empty(4 * K)
    variants = [("wpb1", {"AGN_PRUNE_WPB": "1", "AGN_PRUNE_TAIL_MINW": "1"}),
                ("wpb4", {"AGN_PRUNE_WPB": "4", "AGN_PRUNE_TAIL_MINW": "1"}),
                ("minw8", {"AGN_PRUNE_WPB": "1", "AGN_PRUNE_TAIL_MINW": "8"}),
                ("kpw2", {"AGN_PRUNE_WPB": "1", "AGN_PRUNE_TAIL_KPW": "2"}),
                ("kpw4", {"AGN_PRUNE_WPB": "1", "AGN_PRUNE_TAIL_KPW": "4"})]
    ms = {v: [] for v, _ in variants}
    sig = {}
    for r in range(rounds + 1):
        for name, env in (variants if r % 2 == 0 else variants[::-1]):
            os.environ.update({"AGN_PRUNE_TAIL_KPW": "1", **env})
            env_changed()
            with OpLog(eng, _abi.COUNTER_PN, D, K, init_slots=N + 8) as ol:
                ol.append(keys, oc, txid=txid, eff=eff)
                ol.flush()
                eng.sync()
                b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                b.record()
                ol.prune(bp.ptr, bt.ptr, None, fl.ptr)
                e.record()
                st = ol.stats()
                torch.cuda.synchronize()
                if r:  # round 0 warms both variants up
                    ms[name].append(b.elapsed_time(e))
                print(f"# round {r} {name}: {b.elapsed_time(e):.3f} ms", flush=True)
                if r == 0:
                    ln, lc, ctr = ol.key_meta()
                    sig[name] = (int(st["entries"]), int(ln.astype(np.int64).sum()),
                                 int(np.bitwise_xor.reduce(lc.astype(np.uint64))))
    print(json.dumps({"keys": K, "ops_per_key": N,
                      "gpu_ms_median": {k: float(np.median(v)) for k, v in ms.items()},
                      "gpu_ms_all": ms, "outputs_equal": len(set(sig.values())) == 1,
                      "note": "GPU span of the prune call: k_prune_tail + the records' copy"}),
          flush=True)


if __name__ == "__main__":
    main()
