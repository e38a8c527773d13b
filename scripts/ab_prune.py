"""A/B of the one-pass prune kernel (agn_prune_ops segmented form, the kernel
agn_oplog_prune runs in place) on the cfg2 log, variants alternated in one
process (process-to-process HBM variance is several %):
  round 3: row-slice loads vs contiguous rows (AGN_PRUNE_CT = 0 | 1), and
  the next iteration's rows prefetched (AGN_PRUNE_PF = 0 | 1 | 2; 3: and its
  fields when the iteration before kept everything), the
  register budget of 6 / 8 waves per SIMD (AGN_PRUNE_MINW); round
  2: AGN_PRUNE_WPB = 1 | 4 (waves per block) x AGN_PRUNE_LATE_FIELDS = 0 | 1
  (entry fields with the rows, or only for kept entries after the filter).
  Earlier runs also compared AGN_XCD_REMAP and non-temporal row loads /
  stores (no effect, removed): profiles/r02/ab_prune_*.log.

  python scripts/ab_prune.py [config] [rounds]
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from antidote_amd._lib import env_changed  # noqa: E402


def main():
    import torch
    from antidote_amd import _abi
    from antidote_amd.engine import DeviceArrays, Engine
    from bench import CONFIGS
    config = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    cfg = CONFIGS[config]
    D, N, K = cfg["n_dcs"], cfg["ops_per_key"], cfg["n_keys"]
    E = K * N
    torch.cuda.init()
    eng = Engine(0)
    g = _abi.AgnGenCfg(crdt_type=cfg["crdt_type"], n_dcs=D, n_keys=K, ops_per_key=N,
                       n_elems=cfg["n_elems"], seed=cfg["seed"], key_base=0, key_stride=1, warm=0)
    dl, dr = eng.gen_dev(g)
    s = _abi.AgnLog()
    s.crdt_type, s.n_dcs, s.n_keys, s.n_entries = cfg["crdt_type"], D, K, E
    out = DeviceArrays(s)
    spec = {"key_off": 8 * (K + 1), "oc": 8 * E * D, "op_id": 4 * E, "txid": 8 * E,
            "key_len": 8 * K}
    if cfg["crdt_type"] == 1:
        spec["eff"] = 8 * E
    else:
        n_rem = int(eng.download(type("B", (), {"ptr": dl.rem_off})(), np.uint32, (E + 1,))[-1])
        spec.update({"tag": 4 * E, "add_tok": 8 * E, "rem_off": 4 * (E + 1),
                     "rem_tok": 8 * max(n_rem, 1)})
    for name, nb in spec.items():
        out.bufs[name] = eng.empty(nb)
        setattr(s, name, out.bufs[name].ptr)
    din = DeviceArrays(dl)
    # round 3: row-slice loads vs contiguous rows (AGN_PRUNE_CT), and the
    # next iteration's rows prefetched (AGN_PRUNE_PF; 2 = held to 5 waves)
    variants = [("rows", {"AGN_PRUNE_CT": "0", "AGN_PRUNE_PF": "0", "AGN_PRUNE_MINW": "1"}),
                ("ct", {"AGN_PRUNE_CT": "1", "AGN_PRUNE_PF": "0", "AGN_PRUNE_MINW": "1"}),
                ("pf4", {"AGN_PRUNE_CT": "0", "AGN_PRUNE_PF": "1", "AGN_PRUNE_MINW": "1"}),
                ("pf_ef", {"AGN_PRUNE_CT": "0", "AGN_PRUNE_PF": "3", "AGN_PRUNE_MINW": "1"}),
                ("mw6", {"AGN_PRUNE_CT": "0", "AGN_PRUNE_PF": "0", "AGN_PRUNE_MINW": "6"}),
                ("mw8", {"AGN_PRUNE_CT": "0", "AGN_PRUNE_PF": "0", "AGN_PRUNE_MINW": "8"})]
    os.environ["AGN_PRUNE_WPB"] = "1"
    env_changed()
    best = {v[0]: [] for v in variants}
    sums = {}
    chk = ["key_len", "oc", "op_id"] + (["eff"] if cfg["crdt_type"] == 1 else ["tag", "add_tok", "rem_tok"])
    for r in range(rounds):
        for name, env in (variants if r % 2 == 0 else variants[::-1]):
            os.environ.update(env)
            env_changed()
            eng.prune_ops(din, None, dr.R, None, out)
            torch.cuda.synchronize()
            b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            b.record()
            eng.prune_ops(din, None, dr.R, None, out)
            e.record()
            torch.cuda.synchronize()
            best[name].append(b.elapsed_time(e))
            print(f"# round {r} {name}: {b.elapsed_time(e):.3f} ms", flush=True)
            if r == 0:  # the variants' outputs must be identical
                sig = []
                for c in chk:
                    nb = out.bufs[c].nbytes if hasattr(out.bufs[c], "nbytes") else spec[c]
                    a = eng.download(out.bufs[c], np.uint8, (nb // 8 * 8,)).view(np.uint64)
                    sig.append(int(np.bitwise_xor.reduce(a)) if a.size else 0)
                sums[name] = tuple(sig)
    print(json.dumps({"config": config, "ms_median": {k: float(np.median(v)) for k, v in best.items()},
                      "ms_all": best, "outputs_equal": len(set(sums.values())) == 1}), flush=True)


if __name__ == "__main__":
    main()
