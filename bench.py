#!/usr/bin/env python3
"""bench.py — materialized ops/s (+ VC compares/s) of the MI355X engine.

One step = one agn_materialize pass over the whole device-resident batch: for
every key of this GPU's vnode partitions, the VC snapshot filter + CRDT effect
fold of clocksi_materializer:materialize/4.  Inputs (op log, read clocks) are
generated on the device before the timed region (synthetic, SplitMix64,
BASELINE.md §3); nothing is cached between steps — every step re-reads the
whole log from HBM and rewrites every output.

Sharding (weak scaling): key k lives in partition p = k mod 64 and on GPU
g = p mod G (src/log_utilities.erl:65-70); with G | 64 each rank owns keys
k = rank + G*i, i < keys_per_gpu.  Materialize has no collective.

Default (no flags): N=1, BASELINE cfg2 = counter_pn, 10M keys x 64 ops/key,
8-DC clocks, random snapshot VCs.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4]
  python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)

CONFIGS = {
    1: dict(name="cfg1 counter_pn materialize: {keys} keys x 100 ops/key, 3-DC clocks, random "
                 "snapshot VCs (the reference's CPU-runnable case)", crdt_type=1, n_dcs=3,
            n_keys=10_000, ops_per_key=100, n_elems=0, seed=20250112 + 0),
    2: dict(name="cfg2 counter_pn materialize: {keys} keys x 64 ops/key, 8-DC clocks, "
                 "random snapshot VCs", crdt_type=1, n_dcs=8, n_keys=10_000_000,
            ops_per_key=64, n_elems=0, seed=20250112 + 1),
    3: dict(name="cfg3 set_aw materialize: {keys} keys x 256 add/remove ops, 16-DC clocks, "
                 "32 elems/key, order-aware tag resolution", crdt_type=2, n_dcs=16,
            n_keys=1_000_000, ops_per_key=256, n_elems=32, seed=20250112 + 2),
    5: dict(name="cfg5 GST: 4096 partitions x 256-DC clocks (4096/G per GPU), 256 epochs per step, "
                 "stable_time_functions:get_min_time elementwise min + RCCL ncclMin allreduce "
                 "over xGMI (N > 1)", crdt_type=0, n_dcs=256, n_keys=4096, ops_per_key=0,
            n_elems=0, seed=20250112 + 4, strong=True),
    4: dict(name="cfg4 register_mv materialize: {keys} keys x 100 ops on this GPU (100M ops total over G GPUs), "
                 "64-DC clocks, concurrent-write pruning", crdt_type=3, n_dcs=64,
            n_keys=1_000_000, ops_per_key=100, n_elems=16, seed=20250112 + 3, strong=True),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--keys", type=int, default=0, help="override keys per GPU")
    ap.add_argument("--cpu-keys", type=int, default=-1,
                    help="CPU-baseline sample size in keys (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="extra multi-thread CPU run")
    ap.add_argument("--tune-rounds", type=int, default=3,
                    help="agn_tune launches per kernel variant before timing (0 = no tuning)")
    ap.add_argument("--gst", action="store_true",
                    help="also time a GST epoch + RCCL min-allreduce (always on for N > 1)")
    ap.add_argument("--post-gc", action="store_true",
                    help="also time materialize of a pruned log (op ids with gaps, so the "
                         "NewLastOp id comes from the op_id array instead of key_id0)")
    ap.add_argument("--warm", action="store_true",
                    help="also time the warm read path through the device snapshot cache "
                         "(agn_ss_lookup -> agn_materialize -> agn_ss_store)")
    ap.add_argument("--ingest", action="store_true",
                    help="also time the log-read / recovery ingest (agn_log_ingest) of a "
                         "synthetic partition log")
    ap.add_argument("--gc", action="store_true",
                    help="also time the op-log GC (agn_prune_ops) over the whole log")
    ap.add_argument("--sparse", default="",
                    help="presence masks on every clock (the log the Erlang NIF builds): "
                         "'full' = every DC in every clock, 'subsetN' = the first N DCs in every "
                         "clock (a partition of width D with N interned DCs), 'mixed' = 1 op in 8 "
                         "lacks one random DC (genuinely sparse clocks); counter_pn configs")
    ap.add_argument("--e2e", action="store_true",
                    help="also time the host-staged read path (keys + R from pinned host "
                         "memory, results back to pinned host memory; PCIe-inclusive)")
    ap.add_argument("--configs", default="auto",
                    help="BASELINE configs measured after the headline and reported in the same "
                         "line's 'configs' object: comma list of 1, 2:full, 2:mixed, 3, 4, 5, "
                         "N:warm (read/6 from the device snapshot cache: lookup -> warm "
                         "materialize -> store), N:gc (the one-pass prune_ops GC); "
                         "'auto' = " + AUTO_CONFIGS + " (N = 1) or the multi-GPU ones 4, 5 "
                         "(N > 1) when the headline is the default cfg2 run; 'none' = headline only")
    ap.add_argument("--cpu-target-s", type=float, default=10.0,
                    help="seconds of CPU work per thread count in the CPU baseline")
    return ap.parse_args()


def fmt_keys(n):
    for div, suf in ((1_000_000, "M"), (1_000, "k")):
        if n >= div:
            return f"{n / div:g}{suf}"
    return str(n)


# the default run's sub-configs (N = 1): every BASELINE config, the masked
# cfg2 batch the Erlang NIF's partitions run, the warm read/6 of the three
# materialize configs and the one-pass GC of cfg3
AUTO_CONFIGS = "1,2:full,3,4,5,2:warm,3:warm,4:warm,3:gc"

KERNEL_SOURCES = {   # the sources the dominant kernel of each config is built from
    1: ("mat_counter_dense.hip", "counter_scan.hpp", "filter.hpp", "common.hpp"),
    2: ("mat_counter_dense.hip", "counter_scan.hpp", "filter.hpp", "common.hpp"),
    3: ("mat_tags.hip", "cache_dev.hpp", "filter.hpp", "tags_serve.hpp", "common.hpp"),
    4: ("mat_tags.hip", "cache_dev.hpp", "filter.hpp", "tags_serve.hpp", "common.hpp"),
    5: ("gst.hip", "common.hpp"),
    "gc": ("gc.hip", "filter.hpp", "serve.hpp", "common.hpp"),
}


def lib_provenance():
    """The shared library this process loaded: its sha256 prefix, size and
    mtime, and the hash of every HIP source in antidote_amd/csrc plus the
    header -- so a bench line names the exact build it measured."""
    import hashlib
    lib = os.path.join(ROOT, "antidote_amd", "libantidote_gpu.so")
    h = hashlib.sha256()
    with open(lib, "rb") as fh:
        for blk in iter(lambda: fh.read(1 << 20), b""):
            h.update(blk)
    src = hashlib.sha256()
    cdir = os.path.join(ROOT, "antidote_amd", "csrc")
    for f in sorted(os.listdir(cdir)) + ["../../include/antidote_gpu.h"]:
        path = os.path.join(cdir, f)
        if f.endswith((".hip", ".hpp", ".h")) and os.path.isfile(path):
            src.update(os.path.basename(f).encode())
            with open(path, "rb") as fh:
                src.update(fh.read())
    st = os.stat(lib)
    return {"lib_sha16": h.hexdigest()[:16], "lib_bytes": st.st_size,
            "lib_mtime_utc": time.strftime("%Y-%m-%d %H:%M:%S", time.gmtime(st.st_mtime)),
            "csrc_sha16": src.hexdigest()[:16]}


def kernel_src_sha16(config):
    """Hash of the sources the config's dominant kernel is built from; a PMC
    traffic file (profiles/pmc/cfgN.json, scripts/pmc_traffic.py) is only used
    when it was measured on a build of exactly these sources."""
    import hashlib
    h = hashlib.sha256()
    files = [os.path.join(ROOT, "antidote_amd", "csrc", f) for f in KERNEL_SOURCES[config]] + \
        [os.path.join(ROOT, "include", "antidote_gpu.h")]
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def r_jitter(D):
    """The read-clock jitter of the generator (antidote_amd/csrc/gen.hpp):
    R[d] = max(oc of the ops before the cut) + U[0,4000] - J."""
    J = 16000 // D if D >= 8 else 2000
    return f"U[{-J},{4000 - J}]"


def algorithmic_bytes_survey(cfg, n_keys, n_rem=0, n_live=0):
    """SURVEY.md §8(d)'s byte formula, reported beside the kernel's own
    count: counter_pn per op 8D + 12 (OpSSCommit row, effect, u32 op_id), per
    key 32 + 16D; set_aw / register_mv per op 8D + 20 + 8 per removed token,
    12 per live output pair, per key 32 + 16D."""
    D, N = cfg["n_dcs"], cfg["ops_per_key"]
    ops = n_keys * N
    if cfg["crdt_type"] == 1:
        return ops * (8 * D + 12) + n_keys * (32 + 16 * D)
    return ops * (8 * D + 20) + 8 * n_rem + 12 * n_live + n_keys * (32 + 16 * D)


def algorithmic_bytes(cfg, n_keys, n_rem=0, n_live=0, mask_words=0, mask_ops=0):
    """HBM bytes one materialize launch must move.
    Presence masks (--sparse) add the per-request mask words (mask_words: the
    key's DC set, R's mask word, the LastOpCt mask word -- the latter two
    unless a hint spares them) and the per-entry mask word of the keys whose
    entries differ (mask_ops entries)."""
    D, N = cfg["n_dcs"], cfg["ops_per_key"]
    ops = n_keys * N
    if cfg["crdt_type"] == 1:
        per_op = 8 * D + 8                    # OpSSCommit row + effect
        per_key = 8 + 8 * D + 8 * D + 32      # key_off, R, LastOpCt, value/hole/count/flags/err/op_id
        return ops * per_op + n_keys * per_key + 8 * mask_words + 8 * mask_ops
    per_op = 8 * D + 4 + 4 + 8 + 4            # oc, op_id, tag, add_tok, rem_off
    per_key = 8 + 8 * D + 8 * D + 24 + 8 + 4  # key_off, R, LastOpCt, hole/count/flags/err, out_off, out_n
    return (ops * per_op + 8 * n_rem + 12 * n_live + n_keys * per_key + 8 * mask_words +
            8 * mask_ops)


def presence_masks(mode, D, n_ops, n_keys, rng=None, torch=None):
    """The --sparse masks: (oc_mask[n_ops], R_mask[n_keys]) as int64 words,
    torch tensors on the device (torch given) or numpy arrays."""
    full = (1 << D) - 1
    if mode.startswith("subset"):
        full = (1 << int(mode[6:])) - 1
    elif mode not in ("full", "mixed"):
        raise SystemExit(f"--sparse {mode}: want full, mixed or subsetN")
    if torch is not None:
        ocm = torch.full((n_ops,), full, dtype=torch.int64, device="cuda")
        if mode == "mixed":
            g = torch.Generator(device="cuda").manual_seed(20250112)
            drop = torch.rand(n_ops, device="cuda", generator=g) < 0.125
            d = torch.randint(0, D, (n_ops,), device="cuda", generator=g)
            ocm = torch.where(drop, ocm & ~torch.bitwise_left_shift(torch.ones_like(d), d), ocm)
        rm = torch.full((n_keys,), full, dtype=torch.int64, device="cuda")
        return ocm, rm
    ocm = np.full(n_ops, full, np.uint64)
    if mode == "mixed":
        drop = rng.random(n_ops) < 0.125
        d = rng.integers(0, D, n_ops).astype(np.uint64)
        ocm[drop] &= ~(np.uint64(1) << d[drop])
    return ocm.reshape(n_ops, 1), np.full((n_keys, 1), full, np.uint64)


def cpu_baseline(cfg, n_keys, threads, target_s=10.0, sparse="", warm=0):
    """The C oracle (oracle/liboracle.so, a restatement of the Erlang path) on a
    bounded host-generated sample of the same workload.  Each chunk of the
    sample is materialized `reps` times so that the timed CPU work is about
    target_s seconds per thread count (reps from the first chunk's rate)."""
    from antidote_amd import _abi
    from antidote_amd.encode import alloc_result, result_struct
    from antidote_amd.engine import free_gen_host, gen_host
    lib = _abi.bind(C.CDLL(os.path.join(ROOT, "oracle", "liboracle.so")), _abi.ORACLE_PROTOTYPES)
    chunk = min(n_keys, 500_000 if cfg["n_dcs"] <= 16 else 100_000)
    n_chunks = (n_keys + chunk - 1) // chunk
    tcounts = [1] + ([threads] if threads > 1 else [])
    secs = {nt: 0.0 for nt in tcounts}
    work = {nt: 0 for nt in tcounts}
    reps = {nt: 0 for nt in tcounts}
    done = 0
    while done < n_keys:
        k = min(chunk, n_keys - done)
        g = _abi.AgnGenCfg(crdt_type=cfg["crdt_type"], n_dcs=cfg["n_dcs"], n_keys=k,
                           ops_per_key=cfg["ops_per_key"], n_elems=cfg["n_elems"],
                           seed=cfg["seed"], key_base=done, key_stride=1, warm=warm)
        hl, hr = gen_host(g)
        cap = (np.arange(k + 1, dtype=np.uint64) * np.uint64(cfg["ops_per_key"])
               if cfg["crdt_type"] != 1 else None)
        res = alloc_result(k, cfg["n_dcs"], sparse=bool(sparse), cap_off=cap)
        if sparse:  # the same mask mode on the host sample (library arrays stay the library's)
            ocm, rm = presence_masks(sparse, cfg["n_dcs"], int(hl.n_entries), k,
                                     rng=np.random.default_rng(done))
            hl.oc_mask, hr.R_mask = ocm.ctypes.data, rm.ctypes.data
        os_ = result_struct(res)
        for nt in tcounts:
            r = 0
            while True:
                t0 = time.perf_counter()
                rc = lib.oracle_materialize(C.byref(hl), C.byref(hr), C.byref(os_), nt)
                secs[nt] += time.perf_counter() - t0
                assert rc == 0
                work[nt] += k * cfg["ops_per_key"]
                r += 1
                if not reps[nt]:  # first chunk: size the repetitions
                    reps[nt] = max(1, int(np.ceil(target_s / (secs[nt] * n_chunks))))
                if r >= reps[nt]:
                    break
        if sparse:
            hl.oc_mask = hr.R_mask = None
        free_gen_host(hl, hr)
        done += k
    return {nt: work[nt] / secs[nt] for nt in tcounts}, {nt: secs[nt] for nt in tcounts}, reps


def cpu_baseline_gc(cfg, n_keys, target_s=2.0):
    """The C oracle's prune_ops (oracle_prune_ops: check_filter over every
    key, src/materializer_vnode.erl:566-604) on a bounded host-generated
    sample of the same log, each key's read clock R as its threshold, as
    gc_bench runs the device kernel; 1 thread.  Returns (entries/s, seconds,
    passes)."""
    from antidote_amd import _abi
    from antidote_amd.engine import free_gen_host, gen_host
    lib = _abi.bind(C.CDLL(os.path.join(ROOT, "oracle", "liboracle.so")), _abi.ORACLE_PROTOTYPES)
    D, N = cfg["n_dcs"], cfg["ops_per_key"]
    g = _abi.AgnGenCfg(crdt_type=cfg["crdt_type"], n_dcs=D, n_keys=n_keys, ops_per_key=N,
                       n_elems=cfg["n_elems"], seed=cfg["seed"], key_base=0, key_stride=1, warm=0)
    hl, hr = gen_host(g)
    E = int(hl.n_entries)
    tags = cfg["crdt_type"] != 1
    n_rem = int(np.ctypeslib.as_array(C.cast(hl.rem_off, C.POINTER(C.c_uint32)),
                                      (E + 1,))[-1]) if tags else 0
    arrs = {"key_off": np.zeros(n_keys + 1, np.uint64), "oc": np.zeros(E * D, np.uint64),
            "op_id": np.zeros(E, np.uint32)}
    if hl.txid:  # the generator writes TxIds only for some shapes
        arrs["txid"] = np.zeros(E, np.uint64)
    if tags:
        arrs.update(tag=np.zeros(E, np.uint32), add_tok=np.zeros(E, np.uint64),
                    rem_off=np.zeros(E + 1, np.uint32), rem_tok=np.zeros(max(n_rem, 1), np.uint64))
    else:
        arrs["eff"] = np.zeros(E, np.int64)
    out = _abi.AgnLog()
    out.crdt_type, out.n_dcs, out.n_keys = cfg["crdt_type"], D, n_keys
    for name, arr in arrs.items():
        setattr(out, name, arr.ctypes.data)
    secs, passes = 0.0, 0
    while secs < target_s or passes == 0:
        t0 = time.perf_counter()
        rc = lib.oracle_prune_ops(C.byref(hl), None, hr.R, None, C.byref(out), None)
        secs += time.perf_counter() - t0
        assert rc == 0
        passes += 1
    free_gen_host(hl, hr)
    return E * passes / secs, secs, passes


def warm_line(line, w, cfg, n_keys, world, a):
    """A warm sub-line: read/6 served from the device snapshot cache.  value =
    ops/s of agn_read_cached (lookup -> warm materialize -> store, one C-ABI
    call per step); the roofline is the warm materialize kernel's."""
    ops = n_keys * cfg["ops_per_key"] * world
    ms = w["read_cached_ms"]
    kms = w["materialize_ms"]
    alg = w["materialize_algorithmic_bytes"]
    ach = alg / (kms * 1e-3) / 1e9
    line.update(value=ops / (ms * 1e-3), ms_per_step=ms, vc_compares_per_s=2 * ops / (ms * 1e-3))
    line["config"]["workload"] += (", warm read/6 from the device snapshot cache (agn_read_cached: "
                                   "lookup -> materialize from the cached base -> store)")
    line["roofline"] = {
        "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": ach / HBM_PEAK_GBS, "traffic": w.get("materialize_traffic"),
        "traffic_source": w.get("materialize_traffic_source"),
        "kernel": ("k_counter_quad2 (warm materialize, two requests per wave)"
                   if cfg["crdt_type"] == 1 else "k_tags (warm, from the cached states)"),
        "kernel_ms": kms, "algorithmic_bytes": alg, "kernel_src_sha16": kernel_src_sha16(a.config)}
    line["warm"] = w
    return line


def gc_line(line, gc, cfg, n_keys, world, a):
    """A GC sub-line: prune_ops over every key (the one-pass segmented kernel);
    value = op-log entries filtered per second."""
    seg = gc["segmented"]
    E = gc["entries"] * world
    ach = seg["algorithmic_bytes"] / (seg["ms"] * 1e-3) / 1e9
    line.update(value=E / (seg["ms"] * 1e-3), ms_per_step=seg["ms"], vc_compares_per_s=None,
                unit="ops/s", value_note="op-log entries GC-filtered per second")
    line["config"]["workload"] += (", GC: prune_ops / check_filter of every key against its read "
                                   "clock (snapshot_insert_gc, src/materializer_vnode.erl:513-604)")
    line["roofline"] = {
        "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": ach / HBM_PEAK_GBS, "traffic": seg.get("traffic"),
        "traffic_source": seg.get("traffic_source"),
        "kernel": "k_prune_inplace (segmented one pass)", "kernel_ms": seg["ms"],
        "algorithmic_bytes": seg["algorithmic_bytes"], "kernel_src_sha16": kernel_src_sha16("gc"),
        "frac_of_copy_probe": seg.get("frac_of_copy_probe")}
    line["gc"] = gc
    return line


def pmc_traffic(config, n_units, name=None):
    """HBM bytes per launch of the config's dominant kernel from
    profiles/pmc/cfgN.json (scripts/pmc_traffic.py), only when it was measured
    on this build of the kernel's sources and the same units per launch."""
    sha = kernel_src_sha16(config)
    name = name or f"cfg{config}"
    pmc = os.path.join(ROOT, "profiles", "pmc", f"{name}.json")
    if not os.path.exists(pmc):
        return None, f"null: no PMC pass for {name} (profiles/pmc/)"
    with open(pmc) as f:
        p = json.load(f)
    if p.get("n_keys") == n_units and p.get("kernel_src_sha16") == sha:
        return p.get("hbm_bytes_per_launch"), (
            f"profiles/pmc/{name}.json: rocprofv3 FETCH_SIZE x2 + WRITE_SIZE passes of "
            f"{p.get('kernel')} on this kernel build (sources sha {sha}), "
            f"measured {p.get('measured', '?')}")
    return None, (f"null: profiles/pmc/{name}.json was measured on sources "
                  f"{p.get('kernel_src_sha16')} / {p.get('n_keys')} units, this build is "
                  f"{sha} / {n_units} units")


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(a.gpus)))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and "WORLD_SIZE" in os.environ:
        world = int(os.environ["WORLD_SIZE"])
    import torch
    import torch.distributed as dist
    # AGN_BENCH_BACKEND=gloo: rehearsal of the N > 1 path with several ranks on
    # one GPU (RCCL refuses two ranks on one device); the driver's runs use RCCL
    backend = os.environ.get("AGN_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    env = (torch, dist, world, rank, local, backend)
    line = (gst_main if a.config == 5 else materialize_main)(a, *env)
    # the other BASELINE configs, each its own engine (the previous one's HBM
    # freed), its own warmup + barrier-bracketed timed launches, PMC traffic and
    # a short CPU baseline -- reported in the same JSON line, never in `value`
    configs = {}
    for name, cid, sparse, mode in sub_configs(a, world):
        sa = argparse.Namespace(**vars(a))
        sa.config, sa.sparse, sa.keys, sa.configs = cid, sparse, 0, "none"
        sa.gc = sa.warm = sa.ingest = sa.e2e = sa.gst = sa.post_gc = False
        # a warm / gc sub-line reports that path as its own line (line_mode)
        sa.line_mode = mode
        sa.warm, sa.gc = mode == "warm", mode == "gc"
        sa.steps = max(a.steps, 200) if cid == 1 else a.steps
        sa.cpu_target_s = min(a.cpu_target_s, 2.0)
        sa.cpu_keys = 0 if a.cpu_keys == 0 else -2    # -2: the sub-config sample size
        sub = (gst_main if cid == 5 else materialize_main)(sa, *env)
        if rank == 0:
            configs[name] = {k: v for k, v in sub.items()
                             if k not in ("metric", "higher_is_better", "data", "build",
                                          "vs_baseline", "dtype", "n_gpus", "gen_s")}
    if rank == 0:
        if configs:
            line["configs"] = configs
        detail = write_detail(line)
        print(json.dumps(compact_line(line, detail)), flush=True)
    if world > 1:
        dist.destroy_process_group()


# the driver parses the last stdout line from an ~8 KB tail: the final line
# carries the headline's roofline + cpu_baseline in full and one short summary
# per sub-config; everything else (warm / gc / presence / build / samples)
# goes to the detail file named in the line
LINE_MAX_BYTES = 7000
HEAD_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
             "higher_is_better", "scaling", "vs_baseline", "dtype", "data",
             "vc_compares_per_s", "config", "roofline", "cpu_baseline")
ROOF_KEYS = ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "kernel_ms",
             "algorithmic_bytes", "kernel_src_sha16")
CPU_KEYS = ("value", "unit", "cores", "kind", "sample", "value_mt", "mt_threads")


def _short(s, n=160):
    return s if not isinstance(s, str) or len(s) <= n else s[:n - 3] + "..."


def summarize_sub(sub):
    """One sub-config as the final line carries it: kernel, its time and
    roofline fraction, PMC traffic / algorithmic bytes, the step time and
    the CPU baseline's value."""
    roof = sub.get("roofline") or {}
    cpu = sub.get("cpu_baseline") or {}
    alg, traffic = roof.get("algorithmic_bytes"), roof.get("traffic")
    return {"value": sub.get("value"), "unit": sub.get("unit"),
            "ms_per_step": sub.get("ms_per_step"), "kernel": _short(roof.get("kernel"), 60),
            "kernel_ms": roof.get("kernel_ms"), "frac": roof.get("frac"),
            "algorithmic_bytes": alg, "traffic": traffic,
            "traffic_ratio": traffic / alg if traffic and alg else None,
            "cpu_value": cpu.get("value"),
            **({"exchange_verified": sub["exchange_verified"]} if "exchange_verified" in sub else {}),
            "workload": _short(sub.get("config", {}).get("workload"), 120)}


def compact_line(line, detail_path=None):
    """The driver's line (< LINE_MAX_BYTES): the headline's own keys with its
    full roofline and cpu_baseline, plus summarize_sub() per sub-config."""
    out = {k: line[k] for k in HEAD_KEYS if k in line}
    out["config"] = dict(out.get("config", {}))
    if out.get("roofline"):
        roof = {k: line["roofline"][k] for k in ROOF_KEYS if k in line["roofline"]}
        if roof.get("traffic") and roof.get("algorithmic_bytes"):
            roof["traffic_ratio"] = roof["traffic"] / roof["algorithmic_bytes"]
        roof["traffic_source"] = _short(line["roofline"].get("traffic_source"), 120)
        out["roofline"] = roof
    if out.get("cpu_baseline"):
        cpu = {k: line["cpu_baseline"][k] for k in CPU_KEYS if k in line["cpu_baseline"]}
        cpu["sample"] = _short(cpu.get("sample"), 200)
        cpu["erlang"] = "not reproducible offline (no Erlang runtime)"
        out["cpu_baseline"] = cpu
    build = line.get("build") or {}
    out["build"] = {k: build[k] for k in ("lib_sha16", "csrc_sha16") if k in build}
    if line.get("gst"):  # N > 1: the collective's own check and its epoch
        out["gst"] = {k: line["gst"][k] for k in ("exchange", "exchange_verified", "rccl_ranks",
                                                   "epoch_latency_us") if k in line["gst"]}
    if line.get("configs"):
        out["configs"] = {n: summarize_sub(s) for n, s in line["configs"].items()}
    if detail_path:
        out["detail"] = detail_path
    s = json.dumps(out)
    if len(s) > LINE_MAX_BYTES:  # never lose the headline to its sub-lines
        for sub in out.get("configs", {}).values():
            sub.pop("workload", None)
        if len(json.dumps(out)) > LINE_MAX_BYTES:
            out.pop("configs", None)
    return out


def write_detail(line):
    """The full line (every sub-line's warm / gc / presence / build objects)
    as gpurun_out/bench_detail_<time>.json; returns its repo-relative path
    (None if it could not be written)."""
    rel = os.path.join("gpurun_out", time.strftime("bench_detail_%Y%m%dT%H%M%S.json",
                                                   time.gmtime()))
    try:
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        with open(os.path.join(ROOT, rel), "w") as f:
            json.dump(line, f, indent=1)
    except OSError as e:
        print(f"bench: detail not written: {e}", file=sys.stderr)
        return None
    print(f"bench: full detail in {rel}", file=sys.stderr)
    return rel


def sub_configs(a, world):
    """(name, config, sparse, mode) of the configs measured after the headline:
    "N:full|mixed|subsetK" = presence masks, "N:warm" / "N:gc" = that path."""
    spec = a.configs
    if spec == "auto":
        extra = a.gc or a.warm or a.ingest or a.e2e or a.post_gc or a.gst or a.keys
        if a.config != 2 or a.sparse or extra:
            return []
        spec = AUTO_CONFIGS if world == 1 else "4,5"
    if spec == "none":
        return []
    out = []
    for item in spec.split(","):
        cid, _, opt = item.strip().partition(":")
        if opt in ("warm", "gc"):
            out.append((f"cfg{cid}_{opt}", int(cid), "", opt))
        else:
            out.append((f"cfg{cid}" + (f"_masked_{opt}" if opt else ""), int(cid), opt, ""))
    return out


KERNEL_NAME = {1: "k_counter_key", 2: "k_counter_key", 3: "k_tags", 4: "k_tags", 5: "k_gst_cols"}


def materialize_main(a, torch, dist, world, rank, local, backend):
    """One materialize config: returns the bench line (rank 0) or None."""
    from antidote_amd import _abi
    from antidote_amd.engine import Engine

    cfg = dict(CONFIGS[a.config])
    n_keys = a.keys or cfg["n_keys"]
    if cfg.get("strong") and not a.keys:
        n_keys = cfg["n_keys"] // world      # cfg4 is quoted as a fixed total
    gcfg = _abi.AgnGenCfg(crdt_type=cfg["crdt_type"], n_dcs=cfg["n_dcs"], n_keys=n_keys,
                          ops_per_key=cfg["ops_per_key"], n_elems=cfg["n_elems"],
                          seed=cfg["seed"], key_base=rank, key_stride=world, warm=0)
    eng = Engine(local)
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    t_gen = time.perf_counter()
    dl, dr = eng.gen_dev(gcfg)
    t_gen = time.perf_counter() - t_gen
    cap = None
    if cfg["crdt_type"] != 1:
        cap = np.arange(n_keys + 1, dtype=np.uint64) * np.uint64(cfg["ops_per_key"])
    presence = None
    if a.sparse:
        # presence masks on every clock, as the Erlang NIF's partition logs
        # carry them; agn_log.key_mask as the engine-owned op log maintains it
        ocm_t, rm_t = presence_masks(a.sparse, cfg["n_dcs"], int(dl.n_entries), n_keys,
                                     torch=torch)
        dl.oc_mask, dr.R_mask = ocm_t.data_ptr(), rm_t.data_ptr()
        kmask = eng.index_masks(dl, sp)
        km = eng.download(kmask, np.uint64, (n_keys,), stream=sp)
        mixed = int((km == 0).sum())
        # the promises the read batcher makes for such a batch (agn_read.hints):
        # R masks that carry every DC are not read, a LastOpCt over every
        # column comes back as AGN_F_CT_FULL instead of a mask word
        r_full = not a.sparse.startswith("subset")
        # many keys whose entries differ (> 1/8): scanned in one pass
        many_mixed = mixed * 8 > n_keys
        dr.hints = _abi.HINT_CT_FLAG | (_abi.HINT_R_FULL if r_full else 0) | \
            (_abi.HINT_MIXED if many_mixed else 0)
        # counter_pn reads a mask per entry only for the keys whose entries
        # differ (agn_log.key_mask); the set/register kernel reads every one
        per_entry = mixed if cfg["crdt_type"] == 1 else n_keys
        presence = {"mode": a.sparse, "key_mask": "agn_log_index_masks",
                    "uniform_keys": n_keys - mixed, "mixed_keys": mixed,
                    "mask_ops": per_entry * cfg["ops_per_key"],
                    "hints": ["AGN_HINT_CT_FLAG"] + (["AGN_HINT_R_FULL"] if r_full else []) +
                             (["AGN_HINT_MIXED"] if many_mixed else []),
                    "r_full": r_full}
    res = eng.alloc_result(n_keys, cfg["n_dcs"], sparse=bool(a.sparse), cap_off=cap)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(a.warmup):
        eng.materialize(dl, dr, res, stream=sp)
    # agn_tune (untimed, like warmup): pick this box's faster of the
    # bit-identical row-load variants of the path, if it has two
    tune = None
    if a.tune_rounds > 0:
        choice, tms = eng.tune(dl, dr, res, stream=sp, rounds=a.tune_rounds)
        if choice >= 0:
            names = ["vgpr_rows", "lds_dma_rows", "quad_rows"]
            forced = os.environ.get("AGN_COUNTER_VARIANT", "")[:1]
            if forced not in ("0", "1", "2"):
                forced = os.environ.get("AGN_COUNTER_GLDS", "")[:1]
            if forced in ("0", "1", "2"):  # the environment overrides the selection
                choice = int(forced)
            tune = {"selected": names[choice],
                    "forced_by_env": forced in ("0", "1", "2"),
                    "best_ms": {n: t for n, t in zip(names, tms) if t > 0},
                    "rounds": a.tune_rounds}
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    # the launch's ctypes arguments converted once, and HIP events on the
    # launch stream around the K timed launches only (an event pair around
    # every launch measured 14.7 us per cfg1 step against 6.8 us without:
    # profiles/r03/first_ovh.log) -- kernel_ms is then the kernel's average
    # duration back to back on its stream
    step = eng.bind_materialize(dl, dr, res, stream=sp)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for s in range(a.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / a.steps
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])

    # sanity: outputs exist and no error flags
    flags = eng.download(res.bufs["flags"], np.uint32, (n_keys,))
    count = eng.download(res.bufs["count"], np.uint32, (n_keys,))
    err_keys = int((flags & (_abi.F_ERR_UNEXPECTED | _abi.F_ERR_CORRUPTED |
                             _abi.F_ERR_CAPACITY)).astype(bool).sum())
    n_rem = n_live = 0
    if cfg["crdt_type"] != 1:
        E = n_keys * cfg["ops_per_key"]
        n_rem = int(eng.download(type("B", (), {"ptr": dl.rem_off})(), np.uint32, (E + 1,))[-1])
        n_live = int(eng.download(res.bufs["out_n"], np.uint64 if False else np.uint32,
                                  (n_keys,)).astype(np.int64).sum())

    ops_step = n_keys * cfg["ops_per_key"] * world
    value = ops_step * a.steps / elapsed
    mask_words = 0
    if presence:
        # per request: the key's DC set; R's mask word unless AGN_HINT_R_FULL
        # (the general kernel over the mixed keys reads it anyway); the
        # LastOpCt mask word unless the result carries AGN_F_CT_FULL
        ct_full = int(((flags & np.uint32(_abi.F_CT_FULL)) != 0).sum())
        presence["ct_full_keys"] = ct_full
        mask_words = n_keys + (presence["mixed_keys"] if presence["r_full"] else n_keys) + \
            (n_keys - ct_full)
    bytes_launch = algorithmic_bytes(cfg, n_keys, n_rem, n_live, mask_words,
                                     presence["mask_ops"] if presence else 0)
    bytes_survey = algorithmic_bytes_survey(cfg, n_keys, n_rem, n_live)
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9

    probe = probe_read_gbs(eng, dl, n_keys * cfg["ops_per_key"] * cfg["n_dcs"] * 8, sp, torch)

    gc = gc_bench(eng, dl, dr, cfg, n_keys, sp, torch, a.config) if a.gc else None
    warm = warm_bench(eng, dl, dr, cfg, n_keys, sp, torch, a.steps, a.config) if a.warm else None
    ingest = ingest_bench(eng, cfg, sp, torch) if a.ingest else None
    e2e = e2e_bench(eng, dl, dr, res, cfg, n_keys, torch) if a.e2e else None

    # N > 1: the GST epoch (local min -> RCCL min-allreduce -> finalize) always
    # runs, untimed by the headline, so the scaling run exercises the collective
    gst = None
    if a.gst or world > 1:
        gst = gst_bench(eng, torch, dist, world, rank, sp, backend)
    post_gc = post_gc_bench(eng, cfg, n_keys, rank, world, sp, torch, a.steps) if a.post_gc else None

    line = None
    if rank == 0:
        cpu = None
        # ~64M ops of host-generated sample (8M for a sub-config), timed for
        # ~cpu_target_s seconds per thread count
        n_cpu = a.cpu_keys if a.cpu_keys >= 0 else \
            (64_000_000 if a.cpu_keys == -1 else 8_000_000) // cfg["ops_per_key"]
        mode = getattr(a, "line_mode", "")
        if world == 1 and n_cpu > 0 and mode == "gc":
            n_gc = min(n_keys, max(1, 2_000_000 // cfg["ops_per_key"]))
            rate, secs, passes = cpu_baseline_gc(cfg, n_gc, target_s=a.cpu_target_s)
            cpu = {"value": rate, "unit": "ops/s", "cores": 1, "kind": "port",
                   "sample": f"{n_gc} keys x {cfg['ops_per_key']} ops of the same log "
                             f"(host-generated), oracle_prune_ops (oracle/oracle.c -O3), "
                             f"1 thread, {passes} pass(es) = {secs:.1f} s",
                   "erlang": "not reproducible offline (no Erlang runtime; SURVEY.md §8(c))"}
        elif world == 1 and n_cpu > 0:
            thr = a.cpu_threads or min(16, os.cpu_count() or 1)
            rates, secs, reps = cpu_baseline(cfg, min(n_cpu, n_keys), thr,
                                             target_s=a.cpu_target_s, sparse=a.sparse,
                                             warm=1 if mode == "warm" else 0)
            cpu = {"value": rates[1], "unit": "ops/s", "cores": 1, "kind": "port",
                   "sample": f"{min(n_cpu, n_keys)} keys x {cfg['ops_per_key']} ops of the same "
                             f"workload (host-generated, same SplitMix64 streams), "
                             f"oracle/oracle.c -O3, 1 thread, {reps[1]} pass(es) = "
                             f"{secs[1]:.1f} s of CPU time",
                   "value_mt": rates.get(thr), "mt_threads": thr if thr > 1 else None,
                   "erlang": "not reproducible offline (no Erlang runtime; SURVEY.md §8(c))"}
            if mode == "warm":
                cpu["sample"] += (" -- the warm materialize/4 (SCT = a cached base covering a "
                                  "random prefix); the cache lookup / store are not in it")
        traffic, traffic_src = pmc_traffic(a.config, n_keys,
                                           f"cfg{a.config}_sparse_{a.sparse}" if a.sparse else None)
        kname = KERNEL_NAME[a.config]
        if (not a.sparse and cfg["crdt_type"] == 1 and cfg["n_dcs"] == 8 and
                (tune is None or tune["selected"] == "quad_rows")):
            # dense D = 8 batches run quad rows two requests per wave
            kname = "k_counter_quad2 (two requests per wave)"
        if a.sparse and cfg["crdt_type"] == 1 and cfg["n_dcs"] == 8 and not many_mixed:
            # the masked D = 8 batch: chunk 0 issued under the key's metadata,
            # keys whose entries differ handed to a list pass (empty here)
            kname = "k_counter_q8e2 (two requests per wave; + k_counter_q8m)"

        workload = cfg["name"].format(keys=fmt_keys(n_keys))
        if a.sparse:
            workload += f", presence masks on every clock ({a.sparse})"
        line = {
            "metric": "materialized ops/sec + VC compares/sec (1/2/4/8 GPU), % of HBM roofline",
            "value": value, "unit": "ops/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True, "scaling": "strong" if cfg.get("strong") else "weak",
            "vs_baseline": None, "dtype": "u64",
            "data": "synthetic (device SplitMix64 generator, BASELINE.md §3)",
            "vc_compares_per_s": value,  # SCT = ignore: one D-wide compare per op
            "config": {"workload": workload, "keys_per_gpu": n_keys,
                       "keys_total": n_keys * world,
                       "ops_per_key": cfg["ops_per_key"], "n_dcs": cfg["n_dcs"],
                       "r_jitter": r_jitter(cfg["n_dcs"]),
                       "partitioning": "vnode p = key mod 64, gpu = p mod G; no collective",
                       "parallelism": f"dp{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": traffic_src, "kernel": kname,
                         "kernel_ms": kern_ms, "algorithmic_bytes": bytes_launch,
                         "algorithmic_bytes_survey": bytes_survey,
                         "frac_survey_bytes": bytes_survey / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "kernel_src_sha16": kernel_src_sha16(a.config),
                         "probe_read_GBps": probe,
                         "frac_of_probe": achieved / probe if probe else None},
            "cpu_baseline": cpu,
            "kernel_variant": tune,
            "error_keys": err_keys, "mean_included_ops": float(count.mean()),
            "gen_s": t_gen,
            "build": lib_provenance(),
        }
        if presence:
            line["presence"] = presence
        mode = getattr(a, "line_mode", "")
        if mode == "warm" and warm:
            line = warm_line(line, warm, cfg, n_keys, world, a)
            warm = None
        elif mode == "gc" and gc:
            line = gc_line(line, gc, cfg, n_keys, world, a)
            gc = None
        if gst:
            line["gst"] = gst
        if post_gc:
            line["post_gc"] = post_gc
        if gc:
            line["gc"] = gc
        if warm:
            line["warm"] = warm
        if ingest:
            line["ingest"] = ingest
        if e2e:
            line["e2e"] = e2e

    if presence:  # the masks are torch's, not the generator's
        dl.oc_mask = dr.R_mask = dl.key_mask = None
        del ocm_t, rm_t
    eng.free_gen(dl, dr)
    eng.close()
    torch.cuda.empty_cache()
    return line


def ingest_bench(eng, cfg, sp, torch, n_txn=10_000_000, n_keys=1_000_000):
    """logging_vnode recovery ingest (load_from_log -> get_all ->
    filter_terms_for_key) of a synthetic partition log: n_txn transactions of
    2 counter updates + 1 commit each, 4-way interleaved, D = cfg's DCs."""
    from antidote_amd import _abi
    D = cfg["n_dcs"]
    rng = np.random.default_rng(11)
    n = 3 * n_txn
    # transaction t's records: updates at 3t, 3t+1, commit at 3t+2, then the
    # stream of 4 consecutive transactions is interleaved (u u u u u u u u c c c c)
    t = np.arange(n_txn, dtype=np.uint64)
    kind = np.empty(n, np.uint8)
    txid = np.empty(n, np.uint64)
    blk = n_txn // 4 * 4
    idx = np.arange(blk).reshape(-1, 4)
    base = (idx // 4 * 4)[:, :1] * 3
    for j in range(4):  # updates first, then the four commits
        u0 = (base[:, 0] + 2 * j)
        kind[u0], kind[u0 + 1] = 1, 1
        txid[u0], txid[u0 + 1] = t[idx[:, j]], t[idx[:, j]]
        c = base[:, 0] + 8 + j
        kind[c], txid[c] = 2, t[idx[:, j]]
    rest = np.arange(blk, n_txn)
    kind[3 * rest], kind[3 * rest + 1], kind[3 * rest + 2] = 1, 1, 2
    txid[3 * rest] = txid[3 * rest + 1] = txid[3 * rest + 2] = t[rest]
    key = rng.integers(0, n_keys, n).astype(np.uint64)
    cdc = rng.integers(0, D, n).astype(np.uint32)
    ss = (1_700_000_000_000_000 + rng.integers(0, 10 ** 6, (n, D))).astype(np.uint64)
    ct = ss.max(axis=1) + np.uint64(1)
    eff = rng.integers(-1000, 1000, n).astype(np.int64)
    dev = {k: eng.upload(v) for k, v in dict(kind=kind, txid=txid, key=key, commit_dc=cdc,
                                                commit_time=ct, ss=ss, eff=eff).items()}
    r = _abi.AgnLogRecords()
    r.n = n
    for k, b in dev.items():
        setattr(r, k, b.ptr)
    n_upd = 2 * n_txn
    out = {"key_off": eng.empty(8 * (n_keys + 1)), "oc": eng.empty(8 * n_upd * D),
           "op_id": eng.empty(4 * n_upd), "txid": eng.empty(8 * n_upd), "eff": eng.empty(8 * n_upd)}
    o = _abi.AgnLog()
    for k, b in out.items():
        setattr(o, k, b.ptr)
    tot = eng.empty(16)

    def run():
        rc = eng.lib.agn_log_ingest(eng.ctx, C.byref(r), 1, D, n_keys, None, None, 1, C.byref(o),
                                    tot.ptr, sp)
        assert rc == 0, eng.lib.agn_last_error()
    run()
    torch.cuda.synchronize()
    b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    b.record()
    for _ in range(3):
        run()
    e.record()
    torch.cuda.synchronize()
    ms = b.elapsed_time(e) / 3
    emitted = int(eng.download(tot, np.uint64, (2,))[0])
    for bb in list(dev.values()) + list(out.values()) + [tot]:
        bb.free()
    return {"records": n, "ops_out": emitted, "ms": ms, "records_per_s": n / (ms * 1e-3),
            "ops_per_s": emitted / (ms * 1e-3), "n_keys": n_keys, "n_dcs": D}


def e2e_bench(eng, dl, dr, res, cfg, n_keys, torch, chunk=1 << 20, reps=3):
    """Host-staged read path (what the NIF boundary hands over, SURVEY.md
    §8(b)): the request keys and read clocks R start in pinned host memory,
    the results (value, NewLastOp, LastOpCt, Count, flags, error position) end
    in pinned host memory.  Chunks of `chunk` requests flow through a
    two-slot ring on three streams (H2D copy -> agn_materialize -> D2H copy),
    so PCIe transfers in both directions overlap the kernel.  The op log stays
    resident in HBM (engine-owned, as at update/2 time).  Counter only."""
    from antidote_amd import _abi
    if cfg["crdt_type"] != 1:
        return None
    D = cfg["n_dcs"]
    pin = dict(pin_memory=True)
    # host inputs: request i reads key i with the generator's R row
    keys_h = torch.arange(n_keys, dtype=torch.int64).pin_memory()
    R_h = torch.from_numpy(eng.download(type("B", (), {"ptr": dr.R})(), np.uint64,
                                        (n_keys, D)).view(np.int64)).pin_memory()
    out_spec = {"value": 1, "hole": 1, "lastct": D, "count32": 1, "flags32": 1, "err32": 1}
    host = {"value": torch.empty(n_keys, dtype=torch.int64, **pin),
            "hole": torch.empty(n_keys, dtype=torch.int64, **pin),
            "lastct": torch.empty((n_keys, D), dtype=torch.int64, **pin),
            "count32": torch.empty(n_keys, dtype=torch.int32, **pin),
            "flags32": torch.empty(n_keys, dtype=torch.int32, **pin),
            "err32": torch.empty(n_keys, dtype=torch.int32, **pin)}
    dev = torch.device("cuda", torch.cuda.current_device())
    slots = []
    for _ in range(2):
        s = {"keys": torch.empty(chunk, dtype=torch.int64, device=dev),
             "R": torch.empty((chunk, D), dtype=torch.int64, device=dev)}
        for k, w in out_spec.items():
            s[k] = torch.empty((chunk, w) if w > 1 else chunk, dtype=host[k].dtype, device=dev)
        slots.append(s)
    s_in, s_k, s_out = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    n_chunks = (n_keys + chunk - 1) // chunk

    def run():
        ev_comp = [None, None]   # slot's kernel done (input slot reusable)
        ev_out = [None, None]    # slot's results copied out (result slot reusable)
        for c in range(n_chunks):
            sl, s = c % 2, slots[c % 2]
            a, b = c * chunk, min(n_keys, (c + 1) * chunk)
            m = b - a
            with torch.cuda.stream(s_in):
                if ev_comp[sl] is not None:
                    s_in.wait_event(ev_comp[sl])
                s["keys"][:m].copy_(keys_h[a:b], non_blocking=True)
                s["R"][:m].copy_(R_h[a:b], non_blocking=True)
                ev_in = torch.cuda.Event()
                ev_in.record(s_in)
            s_k.wait_event(ev_in)
            if ev_out[sl] is not None:
                s_k.wait_event(ev_out[sl])
            rq = _abi.AgnRead()
            C.memmove(C.addressof(rq), C.addressof(dr), C.sizeof(_abi.AgnRead))
            rq.n_req, rq.keys, rq.R = m, s["keys"].data_ptr(), s["R"].data_ptr()
            rs = _abi.AgnResult()
            rs.value, rs.hole, rs.lastct = (s[k].data_ptr() for k in ("value", "hole", "lastct"))
            rs.count, rs.flags, rs.err_pos = (s[k].data_ptr() for k in ("count32", "flags32",
                                                                         "err32"))
            eng.materialize(dl, rq, rs, stream=s_k.cuda_stream)
            ev_comp[sl] = torch.cuda.Event()
            ev_comp[sl].record(s_k)
            with torch.cuda.stream(s_out):
                s_out.wait_event(ev_comp[sl])
                for k in out_spec:
                    host[k][a:b].copy_(s[k][:m], non_blocking=True)
                ev_out[sl] = torch.cuda.Event()
                ev_out[sl].record(s_out)
        torch.cuda.synchronize()

    run()
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        run()
        times.append(time.perf_counter() - t0)
    ms = float(np.median(times)) * 1e3
    ref = eng.fetch_result(res)
    same = bool(np.array_equal(ref.value, host["value"].numpy()) and
                np.array_equal(ref.hole, host["hole"].numpy()) and
                np.array_equal(ref.lastct.view(np.int64), host["lastct"].numpy()) and
                np.array_equal(ref.count.view(np.int32), host["count32"].numpy()) and
                np.array_equal(ref.flags.view(np.int32), host["flags32"].numpy()))
    up = n_keys * (8 + 8 * D)
    down = n_keys * (8 + 8 + 8 * D + 4 + 4 + 4)
    ops = n_keys * cfg["ops_per_key"]
    return {"ms": ms, "ops_per_s": ops / (ms * 1e-3), "h2d_bytes": up, "d2h_bytes": down,
            "pcie_GBps": (up + down) / (ms * 1e-3) / 1e9, "chunk_keys": chunk,
            "n_chunks": n_chunks, "same_as_device_resident": same,
            "note": "keys + R from pinned host, results to pinned host; 3 streams, 2-slot ring"}


def warm_bench(eng, dl, dr, cfg, n_keys, sp, torch, steps, cfg_id=None):
    """materializer_vnode:read/6 served from the device snapshot cache: one
    priming pass stores each key's snapshot (IsNewSS, >= 5 ops), then every
    timed step is get_from_snapshot_cache (agn_ss_lookup) -> materialize/4
    from the cached base (SCT, base value: the warm filter, two compares per
    op) -> the cache policy (agn_ss_store)."""
    from antidote_amd import _abi
    D = cfg["n_dcs"]
    if cfg["crdt_type"] != 1:
        return warm_bench_tags(eng, dl, dr, cfg, n_keys, sp, torch, steps, cfg_id)
    S = _abi.SNAPSHOT_THRESHOLD
    bufs = {"n": eng.empty(4 * n_keys), "clock": eng.empty(8 * n_keys * S * D),
            "last_op": eng.empty(8 * n_keys * S), "value": eng.empty(8 * n_keys * S),
            "sct": eng.empty(8 * n_keys * D), "ign": eng.empty(n_keys), "base": eng.empty(8 * n_keys),
            "first": eng.empty(n_keys), "status": eng.empty(n_keys), "prune": eng.empty(n_keys),
            "thr": eng.empty(8 * n_keys * D)}
    eng.lib.agn_memset_d(eng.ctx, bufs["n"].ptr, 0, 4 * n_keys, sp)
    c = _abi.AgnSsCache()
    c.n_dcs, c.slots, c.n_keys = D, S, n_keys
    c.n, c.clock, c.last_op, c.value = (bufs[x].ptr for x in ("n", "clock", "last_op", "value"))
    req = _abi.AgnRead()
    C.memmove(C.addressof(req), C.addressof(dr), C.sizeof(_abi.AgnRead))
    req.sct, req.sct_ignore, req.base_value = bufs["sct"].ptr, bufs["ign"].ptr, bufs["base"].ptr
    res = eng.alloc_result(n_keys, D, sparse=False)

    def step():
        eng.ss_lookup(c, n_keys, None, dr.R, None, bufs["sct"].ptr, None, bufs["ign"].ptr,
                      bufs["base"].ptr, bufs["first"].ptr, bufs["status"].ptr, sp)
        eng.materialize(dl, req, res, sp)
        eng.ss_store(c, dl, n_keys, None, bufs["first"].ptr, bufs["status"].ptr, None, res, None,
                     bufs["prune"].ptr, bufs["thr"].ptr, None, sp)
    step()  # priming: absent keys -> empty snapshot -> cold read -> store
    step()
    torch.cuda.synchronize()
    hits = eng.download(bufs["status"], np.uint8, (n_keys,))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    t_lookup = t_mat = t_store = 0.0
    for _ in range(steps):
        ev[0].record()
        eng.ss_lookup(c, n_keys, None, dr.R, None, bufs["sct"].ptr, None, bufs["ign"].ptr,
                      bufs["base"].ptr, bufs["first"].ptr, bufs["status"].ptr, sp)
        ev[1].record()
        eng.materialize(dl, req, res, sp)
        ev[2].record()
        eng.ss_store(c, dl, n_keys, None, bufs["first"].ptr, bufs["status"].ptr, None, res, None,
                     bufs["prune"].ptr, bufs["thr"].ptr, None, sp)
        ev[3].record()
        torch.cuda.synchronize()
        t_lookup += ev[0].elapsed_time(ev[1])
        t_mat += ev[1].elapsed_time(ev[2])
        t_store += ev[2].elapsed_time(ev[3])
    ms = (t_lookup + t_mat + t_store) / steps
    flags = eng.download(res.bufs["flags"], np.uint32, (n_keys,))
    cnt = eng.download(res.bufs["count"], np.uint32, (n_keys,))
    # the same warm step through agn_read_cached on the same cache: its
    # default dispatch (D = 8: the batched kernels from 5M requests) and the
    # fused kernel forced at this size (AGN_READ_CACHED_SPLIT=0)
    dkeys = eng.upload(np.arange(n_keys, dtype=np.uint64))
    t_rc = {}
    from antidote_amd._lib import set_knob
    old_split = os.environ.get("AGN_READ_CACHED_SPLIT")
    for form, split in (("default", old_split), ("fused", "0")):
        set_knob("AGN_READ_CACHED_SPLIT", split)
        t_rc[form] = 0.0
        for i in range(steps + 1):
            ev[0].record()
            eng.read_cached(c, dl, n_keys, dkeys.ptr, dr.R, dr.txid, None, res,
                            bufs["status"].ptr, bufs["prune"].ptr, bufs["thr"].ptr, sp)
            ev[1].record()
            torch.cuda.synchronize()
            if i:
                t_rc[form] += ev[0].elapsed_time(ev[1])
    set_knob("AGN_READ_CACHED_SPLIT", old_split)
    t_fused = t_rc["fused"]
    hits_f = eng.download(bufs["status"], np.uint8, (n_keys,))
    for b in list(bufs.values()) + list(res.bufs.values()) + [dkeys]:
        b.free()
    ops = n_keys * cfg["ops_per_key"]
    # the warm materialize's bytes: the cold kernel's plus the SCT row, its
    # ignore flag and the base value per request
    wbytes = algorithmic_bytes(cfg, n_keys) + n_keys * (8 * D + 1 + 8)
    # PMC bytes of the warm k_counter_quad2 launches (scripts/gpu.sh pmcwarm:
    # the steps launches after the 2 priming ones, before the 4 launches of
    # agn_read_cached's default dispatch, which at 10M requests is batched)
    wtraffic, wsrc = pmc_traffic(cfg_id, n_keys, f"cfg{cfg_id}_warm") if cfg_id else \
        (None, "null: config id not given")
    return {"ms_per_step": ms, "lookup_ms": t_lookup / steps, "materialize_ms": t_mat / steps,
            "materialize_algorithmic_bytes": wbytes,
            "materialize_traffic": wtraffic, "materialize_traffic_source": wsrc,
            "materialize_frac": wbytes / (t_mat / steps * 1e-3) / 8e12,
            "store_ms": t_store / steps, "ops_per_s": ops / (ms * 1e-3),
            "read_cached_ms": t_rc["default"] / steps,
            "fused_ms": t_fused / steps, "fused_ops_per_s": ops / (t_fused / steps * 1e-3),
            "fused_hit_frac": float((hits_f == _abi.SS_HIT).mean()),
            "vc_compares_per_s": 2 * ops / (ms * 1e-3),
            "cache_hit_frac": float((hits == _abi.SS_HIT).mean()),
            "mean_applied_ops": float(cnt.mean()),
            "error_keys": int((flags & (_abi.F_ERR_UNEXPECTED | _abi.F_ERR_CORRUPTED)).astype(bool).sum())}


def warm_bench_tags(eng, dl, dr, cfg, n_keys, sp, torch, steps, cfg_id=None):
    """read/6 of set_aw / register_mv keys from the device snapshot cache
    (materializer_vnode.erl:384-413,466-509: the cached #materialized_snapshot
    value is the full state): the cache carries a state arena, so a hit's base
    state is read by the tags kernel straight from HBM (AGN_SS_STATE
    references) and the store appends the new state to the arena -- no state
    crosses PCIe.  Priming pass = cold read + store; timed steps = lookup ->
    materialize from the cached state -> store, then the same through
    agn_read_cached (the batched kernels)."""
    from antidote_amd import _abi
    D, N = cfg["n_dcs"], cfg["ops_per_key"]
    S = _abi.SNAPSHOT_THRESHOLD
    # a state never holds more pairs than its key has adding entries (<= N)
    cap_off = np.arange(n_keys + 1, dtype=np.uint64) * np.uint64(N)
    arena_cap = 2 * n_keys * N
    bufs = {"n": eng.empty(4 * n_keys), "clock": eng.empty(8 * n_keys * S * D),
            "last_op": eng.empty(8 * n_keys * S), "value": eng.empty(8 * n_keys * S),
            "sct": eng.empty(8 * n_keys * D), "ign": eng.empty(n_keys), "base": eng.empty(8 * n_keys),
            "first": eng.empty(n_keys), "status": eng.empty(n_keys), "prune": eng.empty(n_keys),
            "thr": eng.empty(8 * n_keys * D), "ctl": eng.empty(32),
            "st_tag": eng.empty(4 * arena_cap), "st_tok": eng.empty(8 * arena_cap)}
    eng.lib.agn_memset_d(eng.ctx, bufs["n"].ptr, 0, 4 * n_keys, sp)
    eng.lib.agn_memset_d(eng.ctx, bufs["ctl"].ptr, 0, 32, sp)
    c = _abi.AgnSsCache()
    c.n_dcs, c.slots, c.n_keys = D, S, n_keys
    c.n, c.clock, c.last_op, c.value = (bufs[x].ptr for x in ("n", "clock", "last_op", "value"))
    c.state_tag, c.state_tok, c.state_cap, c.state_ctl = (bufs["st_tag"].ptr, bufs["st_tok"].ptr,
                                                          arena_cap, bufs["ctl"].ptr)
    req = _abi.AgnRead()
    C.memmove(C.addressof(req), C.addressof(dr), C.sizeof(_abi.AgnRead))
    req.sct, req.sct_ignore, req.base_value = bufs["sct"].ptr, bufs["ign"].ptr, bufs["base"].ptr
    req.base_off, req.base_tag, req.base_tok = None, bufs["st_tag"].ptr, bufs["st_tok"].ptr
    res = eng.alloc_result(n_keys, D, sparse=False, cap_off=cap_off)

    def lookup():
        eng.ss_lookup(c, n_keys, None, dr.R, None, bufs["sct"].ptr, None, bufs["ign"].ptr,
                      bufs["base"].ptr, bufs["first"].ptr, bufs["status"].ptr, sp)

    def store():
        eng.ss_store(c, dl, n_keys, None, bufs["first"].ptr, bufs["status"].ptr, None, res, None,
                     bufs["prune"].ptr, bufs["thr"].ptr, None, sp)
    for _ in range(2):  # priming: absent keys -> empty snapshot -> cold read -> store
        lookup()
        eng.materialize(dl, req, res, sp)
        store()
    torch.cuda.synchronize()
    hits = eng.download(bufs["status"], np.uint8, (n_keys,))
    base_pairs = int((eng.download(bufs["base"], np.int64, (n_keys,)).astype(np.uint64)
                      & np.uint64(0xFFFFFF)).sum())  # AGN_SS_STATE_PAIRS
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    t_lookup = t_mat = t_store = 0.0
    for _ in range(steps):
        ev[0].record()
        lookup()
        ev[1].record()
        eng.materialize(dl, req, res, sp)
        ev[2].record()
        store()
        ev[3].record()
        torch.cuda.synchronize()
        t_lookup += ev[0].elapsed_time(ev[1])
        t_mat += ev[1].elapsed_time(ev[2])
        t_store += ev[2].elapsed_time(ev[3])
    ms = (t_lookup + t_mat + t_store) / steps
    flags = eng.download(res.bufs["flags"], np.uint32, (n_keys,))
    cnt = eng.download(res.bufs["count"], np.uint32, (n_keys,))
    n_live = int(eng.download(res.bufs["out_n"], np.uint32, (n_keys,)).astype(np.int64).sum())
    dkeys = eng.upload(np.arange(n_keys, dtype=np.uint64))
    t_rc = 0.0
    for i in range(steps + 1):
        ev[0].record()
        eng.read_cached(c, dl, n_keys, dkeys.ptr, dr.R, dr.txid, None, res,
                        bufs["status"].ptr, bufs["prune"].ptr, bufs["thr"].ptr, sp)
        ev[1].record()
        torch.cuda.synchronize()
        if i:
            t_rc += ev[0].elapsed_time(ev[1])
    hits_rc = eng.download(bufs["status"], np.uint8, (n_keys,))
    ctl = eng.download(bufs["ctl"], np.uint64, (4,))
    E = n_keys * N
    n_rem = int(eng.download(type("B", (), {"ptr": dl.rem_off})(), np.uint32, (E + 1,))[-1])
    for b in list(bufs.values()) + list(res.bufs.values()) + [dkeys]:
        b.free()
    ops = n_keys * N
    # the warm materialize's bytes: the cold kernel's, plus per request the SCT
    # row, its ignore flag and the base reference, and the base pairs read
    wbytes = (algorithmic_bytes(cfg, n_keys, n_rem, n_live) + n_keys * (8 * D + 1 + 8)
              + 12 * base_pairs)
    # PMC bytes of the warm k_tags launches (scripts/gpu.sh pmcwarm: the
    # steps launches before the steps + 1 agn_read_cached ones)
    wtraffic, wsrc = pmc_traffic(cfg_id, n_keys, f"cfg{cfg_id}_warm") if cfg_id else \
        (None, "null: config id not given")
    return {"ms_per_step": ms, "lookup_ms": t_lookup / steps, "materialize_ms": t_mat / steps,
            "materialize_algorithmic_bytes": wbytes,
            "materialize_traffic": wtraffic, "materialize_traffic_source": wsrc,
            "materialize_frac": wbytes / (t_mat / steps * 1e-3) / 8e12,
            "store_ms": t_store / steps, "ops_per_s": ops / (ms * 1e-3),
            "read_cached_ms": t_rc / steps, "read_cached_ops_per_s": ops / (t_rc / steps * 1e-3),
            "read_cached_hit_frac": float((hits_rc == _abi.SS_HIT).mean()),
            "vc_compares_per_s": 2 * ops / (ms * 1e-3),
            "cache_hit_frac": float((hits == _abi.SS_HIT).mean()),
            "base_pairs": base_pairs, "live_pairs": n_live,
            "arena_pairs_used": int(ctl[0]), "arena_overflow": int(ctl[2]),
            "mean_applied_ops": float(cnt.mean()),
            "state_path": "device (cache state arena; AGN_SS_STATE references)",
            "error_keys": int((flags & (_abi.F_ERR_UNEXPECTED | _abi.F_ERR_CORRUPTED |
                                        _abi.F_ERR_CAPACITY)).astype(bool).sum())}


def gc_bench(eng, dl, dr, cfg, n_keys, sp, torch, cfg_id):
    """materializer_vnode GC (prune_ops) over every key of the device log, with
    each key's read snapshot R as the pruning threshold (a snapshot covering a
    random prefix of its ops), both agn_prune_ops output forms:
      csr       -- mark -> 2 scans -> scatter into a compact CSR log (3 passes,
                   kept rows read twice);
      segmented -- out.key_len given: one pass, each key at its input segment
                   start (the kernel agn_oplog_prune runs in place).
    Out-of-place: a second log of the same size."""
    from antidote_amd import _abi
    from antidote_amd.engine import DeviceArrays
    D, N = cfg["n_dcs"], cfg["ops_per_key"]
    E = n_keys * N
    tags = cfg["crdt_type"] != 1
    s = _abi.AgnLog()
    s.crdt_type, s.n_dcs, s.n_keys, s.n_entries = cfg["crdt_type"], D, n_keys, E
    out = DeviceArrays(s)
    spec = {"key_off": 8 * (n_keys + 1), "oc": 8 * E * D, "op_id": 4 * E, "txid": 8 * E}
    if not tags:
        spec["eff"] = 8 * E
    else:
        n_rem = int(eng.download(type("B", (), {"ptr": dl.rem_off})(), np.uint32, (E + 1,))[-1])
        spec.update({"tag": 4 * E, "add_tok": 8 * E, "rem_off": 4 * (E + 1),
                     "rem_tok": 8 * max(n_rem, 1)})
    for name, nb in spec.items():
        b = eng.empty(nb)
        out.bufs[name] = b
        setattr(s, name, b.ptr)
    key_len = eng.empty(8 * n_keys)
    tot = eng.empty(16)
    din = DeviceArrays(dl)
    per_f = 4 + 8 + (16 if tags else 8)          # op_id, txid, effect fields
    res = {}
    for mode in ("csr", "segmented"):
        s.key_len = key_len.ptr if mode == "segmented" else None
        s.key_id0 = None
        eng.prune_ops(din, None, dr.R, None, out, None, tot.ptr, sp)
        torch.cuda.synchronize()
        b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        b.record()
        for _ in range(3):
            eng.prune_ops(din, None, dr.R, None, out, None, tot.ptr, sp)
        e.record()
        torch.cuda.synchronize()
        ms = b.elapsed_time(e) / 3
        kept, kept_rem = (int(x) for x in eng.download(tot, np.uint64, (2,)))
        per_key = 8 + 8 * D + 8 + (8 if mode == "segmented" else 0)  # key_off, thr, len/off out
        # what the operation must move: every OpSSCommit row once (the filter),
        # the kept entries' fields and removal lists read and written, their rows written
        alg = E * 8 * D + kept * per_f * 2 + kept * 8 * D + 16 * kept_rem + n_keys * per_key
        if mode == "csr":
            # the 3-pass form's own traffic: rows + keep byte, keep byte again,
            # kept rows re-read
            moved = E * (8 * D + 1) + E + 2 * kept * (8 * D + per_f) + 16 * kept_rem + \
                8 * 4 * n_keys
        else:
            # counter_pn loads the fields with the rows (dropped entries' too);
            # set_aw / register_mv only for kept entries (gc.hip late fields)
            moved = alg + (0 if tags else (E - kept) * per_f)
        res[mode] = {"ms": ms, "kept": kept, "algorithmic_bytes": alg,
                     "frac": alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "bytes_moved_by_design": moved,
                     "frac_of_design_bytes": moved / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
    # the box's read+write ceiling at the segmented kernel's write:read mix
    # (tools/bwprobe.hip k_copy over the same arrays, wq of 4 chunks stored)
    seg = res["segmented"]
    seg["traffic"], seg["traffic_source"] = pmc_traffic("gc", n_keys, f"gc_cfg{cfg_id}")
    rd = E * 8 * D + (E if not tags else kept) * per_f
    wq = max(1, min(4, round(4 * (seg["bytes_moved_by_design"] - rd) / max(rd, 1))))
    cp = probe_copy_gbs(eng, dl.oc, out.bufs["oc"].ptr, E * 8 * D, wq, sp, torch)
    if cp:
        seg["copy_probe_GBps"] = cp
        seg["copy_probe_write_frac"] = wq / 4
        seg["frac_of_copy_probe"] = seg["bytes_moved_by_design"] / (seg["ms"] * 1e-3) / 1e9 / cp
    for bb in list(out.bufs.values()) + [tot, key_len]:
        bb.free()
    return {"entries": E, **res,
            "note": "threshold = each key's read clock R; frac on the algorithmic bytes "
                    "(rows once, kept entries read + written)"}


def post_gc_bench(eng, cfg, n_keys, rank, world, sp, torch, steps):
    """materialize/4 after a GC: the warm-generator log (each key has a base
    snapshot SCT covering a random prefix of its ops) is pruned with SCT as
    the threshold (prune_ops keeps the ops not covered by it, so op ids keep
    gaps), re-indexed (agn_log_index_ids: keys whose kept ids are no longer
    consecutive get AGN_ID0_NONE and the counter kernel loads the NewLastOp id
    from op_id), then read warm (SCT, base) like the unpruned log.  Reports
    both, timed alternately in this process."""
    from antidote_amd import _abi
    from antidote_amd.engine import DeviceArrays
    D, N = cfg["n_dcs"], cfg["ops_per_key"]
    g = _abi.AgnGenCfg(crdt_type=cfg["crdt_type"], n_dcs=D, n_keys=n_keys, ops_per_key=N,
                       n_elems=cfg["n_elems"], seed=cfg["seed"], key_base=rank,
                       key_stride=world, warm=1)
    wl, wr = eng.gen_dev(g, sp)
    E = n_keys * N
    s = _abi.AgnLog()
    s.crdt_type, s.n_dcs, s.n_keys, s.n_entries = cfg["crdt_type"], D, n_keys, E
    out = DeviceArrays(s)
    spec = {"key_off": 8 * (n_keys + 1), "oc": 8 * E * D, "op_id": 4 * E}
    if cfg["crdt_type"] == 1:
        spec["eff"] = 8 * E
    else:
        n_rem = int(eng.download(type("B", (), {"ptr": wl.rem_off})(), np.uint32, (E + 1,))[-1])
        spec.update({"tag": 4 * E, "add_tok": 8 * E, "rem_off": 4 * (E + 1),
                     "rem_tok": 8 * max(n_rem, 1)})
    for name, nb in spec.items():
        out.bufs[name] = eng.empty(nb)
        setattr(s, name, out.bufs[name].ptr)
    tot = eng.empty(16)
    eng.prune_ops(DeviceArrays(wl), None, wr.sct, None, out, None, tot.ptr, sp)
    idx = eng.index_ids(out, sp)
    kept = int(eng.download(tot, np.uint64, (2,), stream=sp)[0])
    none_frac = float((eng.download(idx, np.uint32, (n_keys,), stream=sp) ==
                       _abi.ID0_NONE).mean())
    cap = (np.arange(n_keys + 1, dtype=np.uint64) * np.uint64(N)
           if cfg["crdt_type"] != 1 else None)
    res = eng.alloc_result(n_keys, D, sparse=False, cap_off=cap)
    # post_gc_no_index: the same pruned log without agn_log.key_id0, i.e. every
    # key takes the dependent op_id load of the NewLastOp position
    noidx = _abi.AgnLog()
    C.memmove(C.addressof(noidx), C.addressof(out.struct), C.sizeof(_abi.AgnLog))
    noidx.key_id0 = None
    logs = {"unpruned": wl, "post_gc": out.struct, "post_gc_no_index": noidx}
    for lg in logs.values():
        eng.materialize(lg, wr, res, sp)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    ms = {k: 0.0 for k in logs}
    for _ in range(steps):
        for k, lg in logs.items():
            b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            b.record(stream)
            eng.materialize(lg, wr, res, sp)
            e.record(stream)
            e.synchronize()
            ms[k] += b.elapsed_time(e) / steps
    per_key = 8 + 8 * D + 8 * D + 8 * D + 32 + 8   # + SCT row and base value (warm)
    per_op = 8 * D + 8
    byts = {"unpruned": E * per_op + n_keys * per_key,
            "post_gc": kept * per_op + n_keys * per_key,
            "post_gc_no_index": kept * per_op + n_keys * per_key}
    for b in list(out.bufs.values()) + list(res.bufs.values()) + [tot]:
        b.free()
    eng.free_gen(wl, wr)
    return {k: {"ms": ms[k], "entries": E if k == "unpruned" else kept,
                "ops_per_s": (E if k == "unpruned" else kept) / (ms[k] * 1e-3),
                "algorithmic_bytes": byts[k],
                "frac": byts[k] / (ms[k] * 1e-3) / 1e9 / HBM_PEAK_GBS}
            for k in logs} | {"keys_id0_none_frac": none_frac,
                              "note": "warm reads (SCT + base); post_gc = the same log "
                                      "pruned at SCT, op ids with gaps"}


def probe_copy_gbs(eng, src, dst, nbytes, wq, sp, torch):
    """The box's practical read+write rate: tools/libagn_probe.so k_copy reads
    nbytes and writes wq/4 of them (one-shot 4 KiB waves, 16-B accesses);
    GB/s of bytes read + written."""
    path = os.path.join(ROOT, "tools", "libagn_probe.so")
    if not os.path.exists(path):
        return None
    lib = C.CDLL(path)
    lib.agn_probe_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, C.c_void_p]
    for _ in range(2):
        if lib.agn_probe_copy(src, dst, nbytes, wq, sp) != 0:
            return None
    torch.cuda.synchronize()
    b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    b.record()
    for _ in range(5):
        lib.agn_probe_copy(src, dst, nbytes, wq, sp)
    e.record()
    torch.cuda.synchronize()
    moved = (nbytes // 8192 * 8192) * (1 + wq / 4)
    return moved / (b.elapsed_time(e) / 5 * 1e-3) / 1e9


def probe_read_gbs(eng, dl, nbytes, sp, torch):
    """The box's practical HBM read ceiling: tools/libagn_probe.so streams the
    OpSSCommit array (non-temporal LDS-DMA loads, 4 KiB per wave, every byte
    once: the fastest read idiom measured, profiles/r01/ab_read_probe.log) on
    the same stream; reported beside the spec peak so box-to-box HBM variance can be
    told apart from kernel changes."""
    path = os.path.join(ROOT, "tools", "libagn_probe.so")
    if not os.path.exists(path):
        return None
    lib = C.CDLL(path)
    lib.agn_probe_read.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]
    scratch = eng.empty(64)
    for _ in range(2):
        lib.agn_probe_read(dl.oc, nbytes, scratch.ptr, sp)
    b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    b.record()
    for _ in range(5):
        lib.agn_probe_read(dl.oc, nbytes, scratch.ptr, sp)
    e.record()
    torch.cuda.synchronize()
    scratch.free()
    return (nbytes // 8192 * 8192) / (b.elapsed_time(e) / 5 * 1e-3) / 1e9  # whole 8 KiB blocks


def gst_bench(eng, torch, dist, world, rank, sp, backend="nccl"):
    """cfg5: P=4096 partitions x D=256, local min over this GPU's partitions +
    RCCL ncclMin allreduce; single-epoch latency and batched 256-epoch rate.
    With N > 1 the exchange is agn_gst_allreduce (RCCL over xGMI); under the
    gloo rehearsal backend (several ranks on one GPU, which RCCL refuses) the
    same D+1 words are exchanged through torch.distributed on the host."""
    from antidote_amd import _abi
    from antidote_amd.engine import Engine
    D, P, E = 256, 4096, 256
    Pl = P // world
    rng = np.random.default_rng(7 + rank)
    clocks = (1_700_000_000_000_000 + rng.integers(0, 10 ** 9, (E, Pl, D))).astype(np.uint64)
    dc = eng.upload(clocks)
    out = eng.empty(E * (D + 1) * 8)
    rccl = world > 1 and backend == "nccl"
    if rccl:
        uid = [Engine.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        eng.comm_init(world, rank, uid[0])

    def exchange():
        if rccl:
            eng.gst_allreduce(out.ptr, D + 1, sp)
        elif world > 1:
            v = eng.download(out, np.uint64, (D + 1,), stream=sp)
            t = torch.from_numpy(v.view(np.int64).copy())
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            buf = t.numpy().view(np.uint64)
            eng.lib.agn_memcpy_h2d(eng.ctx, out.ptr, buf.ctypes.data, buf.nbytes, sp)
            eng.sync(sp)

    def one(defined=None):
        eng.gst_min(D, Pl, 1, dc.ptr, defined, out.ptr, sp)
        exchange()
        eng.gst_finalize(D, 1, out.ptr, sp)

    for _ in range(5):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        one()
    torch.cuda.synchronize()
    lat = (time.perf_counter() - t0) / 50
    # proof that the exchange combined every rank: the epoch's result must
    # equal the min of every rank's local minima gathered through
    # torch.distributed, then the "some partition undefined => 0" rule
    # (stable_time_functions.erl:78-84) with one undefined partition on the
    # last rank, so the flag word crosses ranks
    verified = None
    if world > 1:
        verified = True
        for undef_rank in (None, world - 1):
            defined = np.ones(Pl, np.uint8)
            if rank == undef_rank:
                defined[Pl // 2] = 0
            ddef = eng.upload(defined)
            eng.gst_min(D, Pl, 1, dc.ptr, ddef.ptr, out.ptr, sp)
            torch.cuda.synchronize()
            local = eng.download(out, np.uint64, (D + 1,), stream=sp).copy()
            exchange()
            eng.gst_finalize(D, 1, out.ptr, sp)
            torch.cuda.synchronize()
            got = eng.download(out, np.uint64, (D + 1,), stream=sp)
            t = torch.from_numpy(local.view(np.int64).copy())   # clocks < 2^63
            if backend == "nccl":
                t = t.cuda()
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            want = t.cpu().numpy().view(np.uint64).copy()
            if want[D] == 0:
                want[:D][want[:D] != np.uint64(_abi.U64_MAX)] = 0
            verified = verified and bool(np.array_equal(got, want)) and \
                (bool(want[D] == 0) == (undef_rank is not None))
            ddef.free()
    b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    eng.gst_min(D, Pl, E, dc.ptr, None, out.ptr, sp)
    b.record()
    for _ in range(5):
        eng.gst_min(D, Pl, E, dc.ptr, None, out.ptr, sp)
    e.record()
    torch.cuda.synchronize()
    ms = b.elapsed_time(e) / 5
    byts = E * Pl * D * 8 + E * (D + 1) * 8
    dc.free()
    out.free()
    return {"epoch_latency_us": lat * 1e6, "batched_epochs": E, "batched_ms": ms,
            "batched_GBps": byts / (ms * 1e-3) / 1e9, "partitions_per_gpu": Pl, "n_dcs": D,
            "exchange": ("rccl" if rccl else "torch.distributed " + backend) if world > 1
            else None,
            "rccl_ranks": world if rccl else None,
            "exchange_verified": verified,
            "epoch": "agn_gst_min -> exchange (min, D+1 words) -> agn_gst_finalize"}


def gst_main(a, torch, dist, world, rank, local, backend):
    """cfg5 as the measured workload: a step is one batch of E = 256 GST
    epochs -- agn_gst_min over this GPU's 4096/G partition clocks for every
    epoch, one exchange of the E x (D+1) words (RCCL ncclMin allreduce over
    xGMI for N > 1, agn_gst_allreduce), agn_gst_finalize.  value = partition
    clock compares per second (P x E per step, whole job: one D-wide
    vectorclock compare per partition per epoch)."""
    from antidote_amd import _abi
    from antidote_amd.engine import Engine
    cfg = CONFIGS[5]
    D, P, E = cfg["n_dcs"], cfg["n_keys"], 256
    Pl = P // world
    eng = Engine(local)
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    gen = torch.Generator(device="cuda")
    gen.manual_seed(cfg["seed"] + rank)
    clocks = (torch.randint(0, 10 ** 9, (E, Pl, D), device="cuda", dtype=torch.int64,
                            generator=gen) + 1_700_000_000_000_000)
    out = torch.empty((E, D + 1), device="cuda", dtype=torch.int64)
    rccl = world > 1 and backend == "nccl"
    if rccl:
        uid = [Engine.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        eng.comm_init(world, rank, uid[0])

    def step(ev=None):
        if ev:
            ev[0].record(stream)
        eng.gst_min(D, Pl, E, clocks.data_ptr(), None, out.data_ptr(), sp)
        if ev:
            ev[1].record(stream)
        if rccl:
            eng.gst_allreduce(out.data_ptr(), E * (D + 1), sp)
        elif world > 1:  # gloo rehearsal: the same words through torch.distributed
            h = out.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.MIN)
            out.copy_(h)
        eng.gst_finalize(D, E, out.data_ptr(), sp)

    def barrier():
        if world > 1:
            dist.barrier()
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(a.steps)]
    t0 = time.perf_counter()
    for s_ in range(a.steps):
        step(evs[s_])
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([b.elapsed_time(e) for b, e in evs]))
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
    # correctness: the exchanged result equals the min over every rank's local vectors
    eng.gst_min(D, Pl, E, clocks.data_ptr(), None, out.data_ptr(), sp)
    torch.cuda.synchronize()
    local_v = out.clone()
    step()
    torch.cuda.synchronize()
    want = local_v.clone()
    if world > 1:
        w = want.cpu() if backend != "nccl" else want
        dist.all_reduce(w, op=dist.ReduceOp.MIN)
        want = w.to(out.device)
    ok = bool(torch.equal(out, want))
    # the "some partition undefined => 0" rule (stable_time_functions.erl:78-84)
    # across ranks: one undefined partition on the last rank
    defined = torch.ones(Pl, device="cuda", dtype=torch.uint8)
    if rank == world - 1:
        defined[Pl // 2] = 0
    one = out[:1]
    eng.gst_min(D, Pl, 1, clocks.data_ptr(), defined.data_ptr(), one.data_ptr(), sp)
    if rccl:
        eng.gst_allreduce(one.data_ptr(), D + 1, sp)
    elif world > 1:
        h = one.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.MIN)
        one.copy_(h)
    eng.gst_finalize(D, 1, one.data_ptr(), sp)
    torch.cuda.synchronize()
    ok = ok and int(one[0, D]) == 0 and bool((one[0, :D] == 0).all())

    # single-epoch latency: one epoch through min -> exchange -> finalize
    def epoch():
        eng.gst_min(D, Pl, 1, clocks.data_ptr(), None, one.data_ptr(), sp)
        if rccl:
            eng.gst_allreduce(one.data_ptr(), D + 1, sp)
        elif world > 1:
            h = one.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.MIN)
            one.copy_(h)
        eng.gst_finalize(D, 1, one.data_ptr(), sp)
    for _ in range(5):
        epoch()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(50):
        epoch()
    torch.cuda.synchronize()
    lat_us = (time.perf_counter() - t1) / 50 * 1e6
    bytes_launch = E * Pl * D * 8 + E * (D + 1) * 8
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
    value = P * E * a.steps / elapsed
    line = None
    if rank == 0:
        traffic, traffic_src = pmc_traffic(5, Pl)
        cpu = None
        if world == 1 and a.cpu_keys != 0:
            lib = _abi.bind(C.CDLL(os.path.join(ROOT, "oracle", "liboracle.so")),
                            _abi.ORACLE_PROTOTYPES)
            Es = 16
            host = np.ascontiguousarray(clocks[:Es].cpu().numpy().view(np.uint64))
            res = np.zeros((Es, D + 1), np.uint64)
            reps, secs = 0, 0.0
            tgt = min(5.0, a.cpu_target_s)
            while secs < tgt:
                t1 = time.perf_counter()
                lib.oracle_gst_min(D, Pl, Es, host.ctypes.data, None, res.ctypes.data, 1)
                secs += time.perf_counter() - t1
                reps += 1
            # N threads: one epoch per thread (ctypes releases the GIL)
            from concurrent.futures import ThreadPoolExecutor
            thr = min(a.cpu_threads or 16, Es)
            row = Pl * D * 8
            def one(e):
                lib.oracle_gst_min(D, Pl, 1, host.ctypes.data + e * row, None,
                                   res.ctypes.data + e * (D + 1) * 8, 1)
            mt_reps, mt_secs = 0, 0.0
            with ThreadPoolExecutor(thr) as ex:
                while mt_secs < tgt:
                    t1 = time.perf_counter()
                    list(ex.map(one, range(Es)))
                    mt_secs += time.perf_counter() - t1
                    mt_reps += 1
            cpu = {"value": P * Es * reps / secs, "unit": "VC compares/s", "cores": 1,
                   "kind": "port", "sample": f"{Es} epochs x {Pl} partitions x {D} DCs, "
                   f"oracle/oracle.c oracle_gst_min -O3, 1 thread, {reps} passes = {secs:.1f} s",
                   "value_mt": P * Es * mt_reps / mt_secs, "mt_threads": thr,
                   "erlang": "not reproducible offline (no Erlang runtime; SURVEY.md §8(c))"}
        line = {
            "metric": "materialized ops/sec + VC compares/sec (1/2/4/8 GPU), % of HBM roofline",
            "value": value, "unit": "VC compares/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic (torch device RNG, clocks near 1.7e15)",
            "config": {"workload": cfg["name"], "partitions_total": P, "partitions_per_gpu": Pl,
                       "n_dcs": D, "epochs_per_step": E, "parallelism": f"dp{world}",
                       "exchange": ("rccl" if rccl else ("torch.distributed " + backend))
                       if world > 1 else None},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": traffic_src, "kernel_src_sha16": kernel_src_sha16(5),
                         "kernel_ms": kern_ms,
                         "kernel": "k_gst_cols",
                         "timed": "agn_gst_min over 256 epochs (k_gst_init + k_gst_cols), HIP events",
                         "algorithmic_bytes": bytes_launch},
            "cpu_baseline": cpu, "exchange_verified": ok, "epoch_latency_us": lat_us,
        }
    del clocks, out
    eng.close()
    torch.cuda.empty_cache()
    return line


if __name__ == "__main__":
    main()
