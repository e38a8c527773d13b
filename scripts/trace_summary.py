"""Average duration of a kernel's full-size launches in a rocprofv3
--kernel-trace CSV (launches >= half the longest one: a bench run also makes
small launches of the same kernel, e.g. cfg5's single-epoch latency loop), to
compare with bench.py's HIP-event kernel_ms.

  python scripts/trace_summary.py <run_kernel_trace.csv> <kernel-substring> [out.json]
"""
import csv
import json
import statistics
import sys


def main():
    path, kern = sys.argv[1], sys.argv[2]
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
         for r in csv.DictReader(open(path)) if kern in r["Kernel_Name"]]
    full = [x for x in d if x >= max(d) / 2]
    rec = {"kernel": kern, "launches": len(d), "full_size_launches": len(full),
           "full_mean_us": statistics.mean(full) / 1e3,
           "full_median_us": statistics.median(full) / 1e3,
           "full_min_us": min(full) / 1e3, "full_max_us": max(full) / 1e3}
    if len(sys.argv) > 3:
        json.dump(rec, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
