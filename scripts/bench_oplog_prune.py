"""Times agn_oplog_prune (engine-owned op log GC) on a synthetic counter log:
K keys x N ops, D = 8 dense clocks (each rep a fresh log) increasing along each key's log, threshold
per key = the clock of a random position, so the ops up to it are pruned.
AGN_LIB selects the library (A/B against tools/libagn_prev.so); AGN_PRUNE_TAIL=0
selects the start-anchored in-place kernel instead of k_prune_tail.

  python scripts/bench_oplog_prune.py [K] [N] [reps]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from antidote_amd import _abi  # noqa: E402
from antidote_amd.engine import Engine, OpLog  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 500_000
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    D = 8
    rng = np.random.default_rng(7)
    keys = np.repeat(np.arange(K, dtype=np.uint64), N)           # appended key-major
    pos = np.tile(np.arange(N, dtype=np.uint64), K)
    oc = (np.uint64(1_700_000_000_000_000) + pos[:, None] * np.uint64(1000)
          + rng.integers(0, 500, (K * N, D), dtype=np.uint64))
    eff = rng.integers(-1000, 1001, K * N, dtype=np.int64)
    txid = np.zeros(K * N, np.uint64)
    cut = rng.integers(0, N, K)
    thr = oc.reshape(K, N, D)[np.arange(K), cut].copy()          # covers ops <= cut (mostly)
    prune = np.ones(K, np.uint8)
    import torch
    torch.cuda.init()
    eng = Engine(0)
    bp, bt = eng.upload(prune), eng.upload(thr)
    fl = eng.empty(4 * K)
    times, call_ms, gpu_ms = [], [], []
    for r in range(reps):
        with OpLog(eng, _abi.COUNTER_PN, D, K, init_slots=N + 8) as ol:
            ol.append(keys, oc, txid=txid, eff=eff)
            ol.flush()
            eng.sync()
            b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            b.record()
            ol.prune(bp.ptr, bt.ptr, None, fl.ptr)     # returns once enqueued
            t1 = time.perf_counter()
            e.record()
            st = ol.stats()                            # settles the host bookkeeping
            times.append((time.perf_counter() - t0) * 1e3)
            call_ms.append((t1 - t0) * 1e3)
            torch.cuda.synchronize()
            gpu_ms.append(b.elapsed_time(e))
    kept = st["entries"]
    ms = float(np.median(times))
    # bytes a start-anchored compaction must move: read every OpSSCommit row
    # (the filter), read the kept entries' effect + id + txid, write them
    per = 8 * D + 8 + 4 + 8
    alg = K * N * 8 * D + kept * (per - 8 * D) + kept * per
    # the end-anchored kernel (k_prune_tail) moves only kept entries with a
    # dropped entry above them: every row read once, movers read + written,
    # per key its metadata (key_off, len, id0, ListLen, threshold; new len,
    # key_off, id0, ListLen, 4 record rows, flag)
    drop = np.all(oc.reshape(K, N, D) <= thr[:, None, :], axis=2)
    above = np.flip(np.logical_or.accumulate(np.flip(drop, 1), 1), 1)
    above = np.concatenate([above[:, 1:], np.zeros((K, 1), bool)], 1)
    moved = int((~drop & above).sum())
    tail = K * N * 8 * D + moved * (2 * per - 8 * D) + K * (24 + 8 * D + 44)
    print(json.dumps({"lib": os.path.basename(os.environ.get("AGN_LIB", "libantidote_gpu.so")),
                      "keys": K, "ops_per_key": N, "n_dcs": D, "kept": int(kept),
                      "ms_median": ms, "ms_all": times,
                      "call_ms_median": float(np.median(call_ms)),
                      "gpu_ms_median": float(np.median(gpu_ms)),
                      "wall_over_gpu": ms / float(np.median(gpu_ms)),
                      "min_bytes": alg, "GBps_min_bytes": alg / ms / 1e6,
                      "GBps_min_bytes_gpu": alg / float(np.median(gpu_ms)) / 1e6,
                      "moved": moved, "tail_bytes": tail,
                      "prune_tail": os.environ.get("AGN_PRUNE_TAIL", "1") != "0",
                      "note": "ms = prune call + settle (stats); gpu_ms = events around the "
                              "prune on its stream (kernel + metadata copy)"}), flush=True)


if __name__ == "__main__":
    main()
