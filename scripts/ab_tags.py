"""A/B of the tag-resolution kernel (k_tags) on the cfg3 / cfg4 shapes, the
variants alternated in one process; every variant's results must equal the
first variant's.

  python scripts/ab_tags.py [ENV=V[,ENV=V...] | base] ...
  e.g. python scripts/ab_tags.py base AGN_TAGS_NT=1
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from antidote_amd._lib import env_changed  # noqa: E402
from antidote_amd import _abi  # noqa: E402
from antidote_amd.engine import Engine  # noqa: E402
from bench import CONFIGS, algorithmic_bytes  # noqa: E402


def parse_variants(args):
    out = []
    for a in args or ["base"]:
        env = {} if a == "base" else dict(kv.split("=", 1) for kv in a.split(","))
        out.append((a, env))
    return out


def main():
    variants = parse_variants(sys.argv[1:])
    knobs = sorted({k for _, env in variants for k in env})
    eng = Engine(0)
    sp = torch.cuda.current_stream().cuda_stream
    report = {}
    for c in (3, 4):
        cfg = CONFIGS[c]
        K = cfg["n_keys"]
        g = _abi.AgnGenCfg(crdt_type=cfg["crdt_type"], n_dcs=cfg["n_dcs"], n_keys=K,
                           ops_per_key=cfg["ops_per_key"], n_elems=cfg["n_elems"],
                           seed=cfg["seed"], key_base=0, key_stride=1, warm=0)
        dl, dr = eng.gen_dev(g)
        cap = np.arange(K + 1, dtype=np.uint64) * np.uint64(cfg["ops_per_key"])
        res = eng.alloc_result(K, cfg["n_dcs"], sparse=False, cap_off=cap)
        E = K * cfg["ops_per_key"]
        n_rem = int(eng.download(type("B", (), {"ptr": dl.rem_off})(), np.uint32, (E + 1,))[-1])
        times = {name: [] for name, _ in variants}
        ref, n_live = None, None
        for rnd in range(8):
            for name, env in (variants if rnd % 2 == 0 else variants[::-1]):
                for k in knobs:
                    os.environ.pop(k, None)
                    env_changed()
                os.environ.update(env)
                env_changed()
                b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                b.record()
                eng.materialize(dl, dr, res, stream=sp)
                e.record()
                torch.cuda.synchronize()
                if rnd >= 2:
                    times[name].append(b.elapsed_time(e))
                if rnd == 0:
                    got = eng.fetch_result(res)
                    fields = ("hole", "lastct", "count", "flags", "out_n", "out_tag", "out_tok")
                    if ref is None:
                        ref = {f: getattr(got, f).copy() for f in fields}
                        n_live = int(got.out_n.astype(np.int64).sum())
                    assert all(np.array_equal(getattr(got, f), ref[f]) for f in fields), name
        byts = algorithmic_bytes(cfg, K, n_rem, n_live)
        report[f"cfg{c}"] = {name: {"ms": float(np.median(t)),
                                    "GBps": byts / float(np.median(t)) / 1e6}
                             for name, t in times.items()}
        eng.free_gen(dl, dr)
        for bb in res.bufs.values():
            bb.free()
    for k in knobs:
        os.environ.pop(k, None)
        env_changed()
    print(json.dumps(report), flush=True)


if __name__ == "__main__":
    main()
