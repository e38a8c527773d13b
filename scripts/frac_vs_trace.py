"""Check every bench line's roofline `kernel_ms` (bench.py's HIP-event timing)
against the same run's rocprofv3 --kernel-trace: the mean duration of the
line's kernel over its full-size launches (>= half the longest launch of
that kernel name: the bench also makes small launches of some kernels, e.g.
cfg2's GST epoch of k_gst_cols).  `frac` is algorithmic bytes / kernel_ms /
peak, so the ratio column is how far each frac is from the trace's.

  python scripts/frac_vs_trace.py <trace.log with the bench JSON line> <run_kernel_trace.csv>
"""
import csv
import json
import statistics
import sys

# bench line -> a substring of its dominant kernel's demangled name
KERNELS = {
    "cfg2": "k_counter_quad2<false, false>",
    "cfg1": "k_counter_key<3,",
    "cfg2_masked_full": "k_counter_q8e2<false",
    "cfg3": "k_tags<4, 4, false, true, true, 256, 1, 2, false, false, true, false",
    "cfg4": "k_tags<4, 16, false, true, false, 256, 1, 2, false, false",
    "cfg5": "k_gst_cols",
    "cfg2_warm": "k_counter_quad2<true, false>",
    "cfg3_warm": "k_tags<4, 4, false, true, true, 256, 1, 2, true, false",
    "cfg4_warm": "k_tags<4, 16, false, true, false, 256, 1, 2, true, false",
    "cfg3_gc": "k_prune_inplace<8, 2, false, true, true",
}


def main():
    line = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
    d = json.loads(line)
    lines = {"cfg2": d}
    lines.update({k: v for k, v in d.get("configs", {}).items() if isinstance(v, dict)})
    rows = list(csv.DictReader(open(sys.argv[2])))
    print(f"{'line':18s} {'bench kernel_ms':>15s} {'trace mean ms':>13s} {'launches':>8s} {'ratio':>6s}  frac")
    for name, pat in KERNELS.items():
        x = lines.get(name)
        if not x:
            continue
        # full sub-lines carry a roofline object; the final line's compact
        # summaries (bench.compact_line) carry kernel_ms / frac directly
        roof = x.get("roofline") or x
        if "kernel_ms" not in roof:
            continue
        dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
               for r in rows if pat in r["Kernel_Name"]]
        if not dur:
            print(f"{name:18s} no trace launches for {pat!r}")
            continue
        full = [t for t in dur if t >= max(dur) / 2]
        km = roof["kernel_ms"]
        mean = statistics.mean(full)
        print(f"{name:18s} {km:15.4f} {mean:13.4f} {len(full):8d} {km / mean:6.3f}  "
              f"{roof['frac']:.3f}")


if __name__ == "__main__":
    main()
