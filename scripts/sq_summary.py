"""Per-kernel averages of a rocprofv3 --pmc counter CSV (SQ_* counters: per
wave and as a fraction of SQ_WAVE_CYCLES), over the launches of at least half
the largest launch's waves.  python scripts/sq_summary.py <run_counter_collection.csv>"""
import csv, sys, collections, re
path = sys.argv[1]
rows = list(csv.DictReader(open(path)))
agg = collections.defaultdict(lambda: collections.defaultdict(dict))
for r in rows:
    k = r["Kernel_Name"]
    m = re.search(r"(k_\w+)(<[^()]*>)?", k)
    name = (m.group(1) + (m.group(2) or "")) if m else k[:50]
    agg[name][r["Counter_Name"]][int(r["Dispatch_Id"])] = float(r["Counter_Value"])
for k, cs in agg.items():
    disp = sorted(set(d for v in cs.values() for d in v))
    big = [d for d in disp if cs.get("SQ_WAVES", cs.get("FETCH_SIZE", {})).get(d, 0) >= 0.5 * max(cs.get("SQ_WAVES", cs.get("FETCH_SIZE", {})).values())]
    if not k.startswith("k_"): continue
    print(k[:110], "dispatches", len(disp), "big", len(big))
    wc = sum(cs["SQ_WAVE_CYCLES"][d] for d in big) / len(big) if "SQ_WAVE_CYCLES" in cs else None
    for c, v in sorted(cs.items()):
        val = sum(v[d] for d in big) / len(big)
        extra = f"  ({val / wc:.3f} of WAVE_CYCLES)" if wc and c.startswith(("SQ_WAIT", "SQ_ACTIVE")) else ""
        per = f"  per wave {val / (sum(cs['SQ_WAVES'][d] for d in big)/len(big)):.1f}" if "SQ_WAVES" in cs and c != "SQ_WAVES" else ""
        print(f"   {c:22s} {val:.4g}{extra}{per}")
