"""scripts/pmc_traffic.py (host logic, no GPU): the per-dispatch values of a
kernel from a rocprofv3 counter CSV -- full-size launches only, in dispatch
order, and the tail:A:B selection the warm PMC recipe uses (the warm
materialize steps before the agn_read_cached launches, scripts/gpu.sh
pmcwarm)."""
import csv
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import pmc_traffic  # noqa: E402


def write_csv(path, rows):
    cols = ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"]
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=cols)
        w.writeheader()
        for r in rows:
            w.writerow(dict(zip(cols, r)))


def test_values_full_size_in_dispatch_order(tmp_path):
    p = str(tmp_path / "fetch.csv")
    # out of order in the file; a small launch (parity check) and another kernel
    write_csv(p, [(3, "k_tags<...>", "FETCH_SIZE", 103.0), (1, "k_tags<...>", "FETCH_SIZE", 101.0),
                  (2, "k_tags<...>", "FETCH_SIZE", 5.0), (4, "k_gen", "FETCH_SIZE", 999.0),
                  (5, "k_tags<...>", "WRITE_SIZE", 7.0), (6, "k_tags<...>", "FETCH_SIZE", 106.0)])
    assert pmc_traffic.values(p, "k_tags", "FETCH_SIZE") == [101.0, 103.0, 106.0]


def test_values_tail_selection(tmp_path):
    p = str(tmp_path / "fetch.csv")
    # cold x4, priming x2, warm x3 (200..202), read_cached x4
    vals = [100.0] * 4 + [150.0] * 2 + [200.0, 201.0, 202.0] + [300.0] * 4
    write_csv(p, [(i + 1, "k_tags", "FETCH_SIZE", v) for i, v in enumerate(vals)])
    assert pmc_traffic.values(p, "k_tags", "FETCH_SIZE", "tail:3:4") == [200.0, 201.0, 202.0]
