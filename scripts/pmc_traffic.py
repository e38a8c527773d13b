"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes (separate runs, one counter
each) into HBM bytes per launch of the dominant kernel, with the gfx950
correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half the bytes of
a wide coalesced stream (x2); WRITE_SIZE is exact for 16-B stores; both in KB.

  python scripts/pmc_traffic.py <fetch.csv> <write.csv> <kernel-substring> <n_keys> <config|gc> <out.json> [tail:A:B]

The record carries the hash of the kernel's sources (bench.kernel_src_sha16),
so bench.py uses it only for a build of exactly those sources.
"""
import os
import time
import csv
import json
import statistics
import sys


def values(path, kern, counter, select=None):
    """Per-dispatch values of the kernel, keeping only the full-size launches
    (>= half the largest): a bench run also makes small launches of the same
    kernel (parity checks, cfg5's single-epoch latency loop).  select =
    "tail:A:B": of those, in dispatch order, the A launches before the last B
    (bench.py --warm: the warm materialize steps come before the steps + 1
    agn_read_cached launches)."""
    rows = []
    for r in csv.DictReader(open(path)):
        if kern in r.get("Kernel_Name", "") and r.get("Counter_Name") == counter:
            rows.append((int(r.get("Dispatch_Id") or 0), float(r["Counter_Value"])))
    rows.sort()
    out = [v for _, v in rows]
    top = max(out)
    out = [v for v in out if v >= 0.5 * top]
    if select:
        _, a, b = select.split(":")
        a, b = int(a), int(b)
        out = out[len(out) - a - b:len(out) - b]
    return out


def main():
    fetch, write, kern, n_keys, config, dst = sys.argv[1:7]
    select = sys.argv[7] if len(sys.argv) > 7 else None
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from bench import kernel_src_sha16
    f = values(fetch, kern, "FETCH_SIZE", select)
    w = values(write, kern, "WRITE_SIZE", select)
    fb = statistics.median(f) * 1024 * 2
    wb = statistics.median(w) * 1024
    rec = {"kernel": kern, "n_keys": int(n_keys), "dispatches": [len(f), len(w)],
           "select": select,
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
