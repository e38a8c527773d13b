"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes (separate runs, one counter
each) into HBM bytes per launch of the dominant kernel, with the gfx950
correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half the bytes of
a wide coalesced stream (x2); WRITE_SIZE is exact for 16-B stores; both in KB.

  python scripts/pmc_traffic.py <fetch.csv> <write.csv> <kernel-substring> <n_keys> <config|gc> <out.json>

The record carries the hash of the kernel's sources (bench.kernel_src_sha16),
so bench.py uses it only for a build of exactly those sources.
"""
import os
import time
import csv
import json
import statistics
import sys


def values(path, kern, counter):
    """Per-dispatch values of the kernel, keeping only the full-size launches
    (>= half the largest): a bench run also makes small launches of the same
    kernel (parity checks, cfg5's single-epoch latency loop)."""
    out = []
    for r in csv.DictReader(open(path)):
        if kern in r.get("Kernel_Name", "") and r.get("Counter_Name") == counter:
            out.append(float(r["Counter_Value"]))
    top = max(out)
    return [v for v in out if v >= 0.5 * top]


def main():
    fetch, write, kern, n_keys, config, dst = sys.argv[1:7]
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from bench import kernel_src_sha16
    f = values(fetch, kern, "FETCH_SIZE")
    w = values(write, kern, "WRITE_SIZE")
    fb = statistics.median(f) * 1024 * 2
    wb = statistics.median(w) * 1024
    rec = {"kernel": kern, "n_keys": int(n_keys), "dispatches": [len(f), len(w)],
           "fetch_size_kb_median": statistics.median(f), "write_size_kb_median": statistics.median(w),
           "hbm_read_bytes_per_launch": fb, "hbm_write_bytes_per_launch": wb,
           "hbm_bytes_per_launch": fb + wb,
           "correction": "FETCH_SIZE x2 (gfx950 wide-stream undercount), KB x1024",
           "kernel_src_sha16": kernel_src_sha16(int(config) if config.isdigit() else config),
           "measured": time.strftime("%Y-%m-%d %H:%M UTC", time.gmtime())}
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    json.dump(rec, open(dst, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
