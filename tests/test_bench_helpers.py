"""bench.py's measurement plumbing on the CPU: the PMC traffic attached to a
bench line is the file measured on exactly the kernel's current sources and
units per launch (scripts/pmc_traffic.py output), never a stale one, and the
algorithmic byte counts follow DESIGN.md §4 / SURVEY.md §8(d)."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_kernel_sha_covers_sources_and_header(tmp_path, monkeypatch):
    base = bench.kernel_src_sha16(2)
    assert len(base) == 16 and base == bench.kernel_src_sha16(2)
    # configs built from the same sources share the hash; others differ
    assert bench.kernel_src_sha16(1) == base
    assert bench.kernel_src_sha16(3) != base and bench.kernel_src_sha16(5) != base
    # any change to one of the sources (or the ABI header) changes it
    fake = tmp_path / "antidote_amd" / "csrc"
    fake.mkdir(parents=True)
    (tmp_path / "include").mkdir()
    for f in bench.KERNEL_SOURCES[2]:
        (fake / f).write_bytes(open(os.path.join(ROOT, "antidote_amd", "csrc", f), "rb").read())
    hdr = open(os.path.join(ROOT, "include", "antidote_gpu.h"), "rb").read()
    (tmp_path / "include" / "antidote_gpu.h").write_bytes(hdr)
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.kernel_src_sha16(2) == base
    (tmp_path / "include" / "antidote_gpu.h").write_bytes(hdr + b"\n")
    assert bench.kernel_src_sha16(2) != base


def test_pmc_traffic_only_on_matching_build(tmp_path, monkeypatch):
    sha = bench.kernel_src_sha16(2)
    pmc = tmp_path / "profiles" / "pmc"
    pmc.mkdir(parents=True)
    # the hash of the real sources; the PMC directory is a scratch one
    monkeypatch.setattr(bench, "kernel_src_sha16", lambda c: sha)
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    v, why = bench.pmc_traffic(2, 10_000_000)
    assert v is None and "no PMC pass" in why
    rec = {"kernel": "k_counter_key", "n_keys": 10_000_000, "hbm_bytes_per_launch": 4.85e10,
           "kernel_src_sha16": sha, "measured": "test"}
    (pmc / "cfg2.json").write_text(json.dumps(rec))
    v, why = bench.pmc_traffic(2, 10_000_000)
    assert v == 4.85e10 and sha in why
    v, why = bench.pmc_traffic(2, 5_000_000)  # other units per launch
    assert v is None and "5000000 units" in why
    (pmc / "cfg2.json").write_text(json.dumps({**rec, "kernel_src_sha16": "0" * 16}))
    v, why = bench.pmc_traffic(2, 10_000_000)
    assert v is None and "0" * 16 in why


@pytest.mark.parametrize("config", [1, 2, 3, 4, 5])
def test_committed_pmc_files_are_well_formed(config):
    p = os.path.join(ROOT, "profiles", "pmc", f"cfg{config}.json")
    d = json.load(open(p))
    assert d["hbm_bytes_per_launch"] > 0 and len(d["kernel_src_sha16"]) == 16
    assert d["n_keys"] == {1: 10_000, 2: 10_000_000, 3: 1_000_000, 4: 1_000_000, 5: 4096}[config]


def test_algorithmic_bytes_match_design():
    """cfg2's per-launch bytes (47.76 GB; SURVEY.md §8(d):
    50.24 GB) and the per-op / per-key terms of the counter formula."""
    c2 = bench.CONFIGS[2]
    assert bench.algorithmic_bytes(c2, 10_000_000) == 47_760_000_000
    assert bench.algorithmic_bytes_survey(c2, 10_000_000) == 50_240_000_000
    c1 = bench.CONFIGS[1]
    D, N, K = c1["n_dcs"], c1["ops_per_key"], c1["n_keys"]
    assert bench.algorithmic_bytes(c1, K) == K * N * (8 * D + 8) + K * (8 + 16 * D + 32)
    # set/register terms grow with removed tokens and live output pairs
    c3 = bench.CONFIGS[3]
    b0 = bench.algorithmic_bytes(c3, 1000)
    assert bench.algorithmic_bytes(c3, 1000, n_rem=10, n_live=5) == b0 + 80 + 60


def test_final_line_fits_driver_tail():
    """The default run's final stdout line, built from a recorded full line
    (round 5's closing run: headline + nine sub-lines, 20.5 KB), stays under
    8000 bytes and keeps the headline's roofline / cpu_baseline whole and one
    summary per sub-config."""
    full = json.load(open(os.path.join(ROOT, "profiles", "r05", "bench_default_closing.json")))
    out = bench.compact_line(full, "gpurun_out/bench_detail_x.json")
    s = json.dumps(out)
    assert len(s) < 8000, len(s)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "dtype", "config"):
        assert out[k] == full[k]
    roof = out["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel_ms",
              "algorithmic_bytes"):
        assert roof[k] == full["roofline"][k]
    assert roof["traffic_ratio"] == pytest.approx(roof["traffic"] / roof["algorithmic_bytes"])
    for k in ("value", "unit", "cores", "kind"):
        assert out["cpu_baseline"][k] == full["cpu_baseline"][k]
    assert set(out["configs"]) == set(full["configs"])
    for name, sub in out["configs"].items():
        src = full["configs"][name]
        assert sub["frac"] == src["roofline"]["frac"]
        assert sub["kernel_ms"] == src["roofline"]["kernel_ms"]
        assert sub["ms_per_step"] == src["ms_per_step"]
        assert sub["cpu_value"] == (src.get("cpu_baseline") or {}).get("value")
    # a line that would not fit drops sub-line detail, never the headline
    big = dict(full, configs={f"c{i}": full["configs"]["cfg3_gc"] for i in range(60)})
    out = bench.compact_line(big)
    assert len(json.dumps(out)) < 8000 and out["roofline"]["frac"] == full["roofline"]["frac"]


def test_final_line_keeps_the_exchange_check():
    """N > 1: the GST exchange's own verification survives the compaction
    (the headline's gst object and cfg5's sub-line)."""
    full = json.load(open(os.path.join(ROOT, "profiles", "r06", "bench_n2_gloo_detail.json")))
    out = bench.compact_line(full)
    assert len(json.dumps(out)) < 8000
    assert out["gst"]["exchange_verified"] is True and out["n_gpus"] == 2
    assert out["configs"]["cfg5"]["exchange_verified"] is True


def test_committed_final_line_is_its_detail_compacted():
    """Round 6's committed final line (profiles/r06/bench_final_line.json, the
    line DESIGN.md §4.8 quotes) is exactly bench.compact_line of the detail
    file the same run wrote, and every sub-line carries PMC traffic."""
    full = json.load(open(os.path.join(ROOT, "profiles", "r06", "bench_final_detail.json")))
    line = json.load(open(os.path.join(ROOT, "profiles", "r06", "bench_final_line.json")))
    assert bench.compact_line(full, line.get("detail")) == line
    assert len(json.dumps(line)) < 8000
    assert line["roofline"]["traffic"] is not None
    assert all(sub.get("traffic") is not None for sub in line["configs"].values())
