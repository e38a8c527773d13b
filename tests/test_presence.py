"""Presence masks on the dense counter kernels (ABI v4, agn_log.key_mask).

The reference's clocks are dicts (include/antidote.hrl:188): a DC missing
from an op's OpSSCommit is not compared, a DC of the op missing from the read
snapshot excludes it (src/clocksi_materializer.erl:245-247), a DC missing
from SCT reads 0, and LastOpCt's DC set is SCT's united with the included
ops' (:249-256).  The Erlang NIF builds every partition log with presence
masks (nif_part_open, sparse = 1), so these are the semantics the drop-in
runs.  Covered here, each against the C oracle (or the reference's ETS
transcription) bit for bit:

  * keys whose entries all carry one DC set U (the steady state: the dense
    row scan with U's columns only) and keys whose entries differ (the
    per-entry-mask scan), mixed in one batch, cold and warm, through every
    counter kernel (VGPR rows, quad rows, two requests per wave, general);
    absent columns hold garbage, present ones sometimes 0;
  * agn_log_index_masks against numpy;
  * a log whose masks are all full equals the dense log;
  * the NIF's call sequence on a sparse engine-owned log (one DC joining
    halfway) equals the same sequence on a dense log and the reference's
    transcription.
"""
import ctypes as C

import numpy as np
import pytest

from antidote_amd import _abi
from antidote_amd.encode import alloc_result, log_struct, read_struct, result_struct
from antidote_amd.engine import Batcher, OpLog
from oracle import py_oracle as po
from synth import compare, random_case

pytestmark = pytest.mark.gpu


def presence_case(seed, K, D, nmax, *, p_uniform=0.7, p_cover=0.85, garbage=True, warm=0.4,
                  crdt=_abi.COUNTER_PN, with_cap=False, **kw):
    """random_case with per-key DC sets: a fraction p_uniform of the keys have
    one DC set U on every entry; R covers U for a fraction p_cover of the
    reads; absent columns of op rows, R and SCT hold garbage."""
    log, req, cap = random_case(seed, crdt, K, D, nmax, sparse=True, warm=warm, **kw)
    rng = np.random.default_rng(seed + 1)
    full = (1 << D) - 1 if D < 64 else (1 << 64) - 1
    keys = req.keys
    inv = np.empty(K, np.int64)
    inv[keys.astype(np.int64)] = np.arange(K)
    for k in range(K):
        a, b = int(log.key_off[k]), int(log.key_off[k + 1])
        i = inv[k]
        if rng.random() < p_uniform:
            U = int(rng.integers(1, min(full, (1 << 62)) + 1))
            log.oc_mask[a:b, 0] = np.uint64(U)
        else:
            U = int(np.bitwise_or.reduce(log.oc_mask[a:b, 0])) if b > a else full
        if rng.random() < p_cover:
            req.R_mask[i, 0] = np.uint64(U | int(rng.integers(0, min(full, (1 << 62)) + 1)))
        # a few present values are 0 (a DC at time 0 is still present)
        z = rng.random((b - a, D)) < 0.02
        log.oc[a:b][z] = 0
    if garbage:
        big = lambda shape: rng.integers(1 << 40, 1 << 62, shape, dtype=np.int64).astype(np.uint64)  # noqa: E731
        bits = ((log.oc_mask[:, :1] >> np.arange(D, dtype=np.uint64)) & np.uint64(1)).astype(bool)
        log.oc[~bits] = big(int((~bits).sum()))
        rb = ((req.R_mask[:, :1] >> np.arange(D, dtype=np.uint64)) & np.uint64(1)).astype(bool)
        req.R[~rb] = big(int((~rb).sum()))
        sb = ((req.sct_mask[:, :1] >> np.arange(D, dtype=np.uint64)) & np.uint64(1)).astype(bool)
        req.sct[~sb] = big(int((~sb).sum()))
    return (log, req, cap) if with_cap else (log, req)


def oracle_result(oracle_lib, log, req, cap=None):
    res = alloc_result(req.n_req, log.n_dcs, sparse=True, cap_off=cap)
    ls, rs, os_ = log_struct(log), read_struct(req, sparse=True), result_struct(res)
    assert oracle_lib.oracle_materialize(C.byref(ls), C.byref(rs), C.byref(os_), 4) == 0
    return res


def device_result(eng, log, req, index, hints=0):
    dl, dr = eng.upload_log(log), eng.upload_read(req, sparse=True)
    dr.struct.hints = hints
    if index:
        eng.index_masks(dl)
    dres = eng.alloc_result(req.n_req, log.n_dcs, sparse=True)
    eng.materialize(dl, dr, dres)
    return eng.fetch_result(dres)


IMPLS = {"vgpr": "0", "quad": "2", "quad2": "3", "split": "2", "split_km1": "2",
         "split_ctflag": "2", "split_mixed": "2", "split_two": "2", "split_cold": "2",
         "split_one_cold": "2"}


@pytest.mark.parametrize("path", ["host", "device_indexed", "device_no_index"])
@pytest.mark.parametrize("impl", ["vgpr", "quad", "quad2", "general", "split", "split_km1",
                                  "split_ctflag", "split_mixed", "split_two", "split_cold",
                                  "split_one_cold"])
@pytest.mark.parametrize("D", [1, 3, 5, 8])
def test_presence_vs_oracle(eng, oracle_lib, monkeypatch, D, impl, path):
    """quad / quad2 / vgpr: k_counter_key (AGN_COUNTER_EARLY=0); split: the
    default masked D = 8 path -- k_counter_q8e with its hand-ons (keys whose
    entries differ) to the list pass k_counter_q8m; _km1 with the key's DC set
    loaded with the segment metadata (AGN_Q8E_KM=1), _ctflag with AGN_HINT_CT_FLAG
    (LastOpCt masks over every column as AGN_F_CT_FULL), _mixed with
    AGN_HINT_MIXED (k_counter_key: the mixed keys in the same pass), _two with
    the warm requests (SCT given) two per wave (k_counter_q8e2,
    AGN_Q8E_TWO=1); _cold a batch without SCT two per wave (q8e2's cold form,
    the default), _one_cold the same batch one per wave (AGN_Q8E_TWO=0)."""
    monkeypatch.delenv("AGN_COUNTER_GLDS", raising=False)
    monkeypatch.setenv("AGN_COUNTER_VARIANT", IMPLS.get(impl, "0"))
    monkeypatch.setenv("AGN_COUNTER_EARLY", "1" if impl.startswith("split") else "0")
    monkeypatch.setenv("AGN_Q8E_KM", "1" if impl == "split_km1" else "0")
    if impl == "split_cold":
        monkeypatch.delenv("AGN_Q8E_TWO", raising=False)
    else:
        monkeypatch.setenv("AGN_Q8E_TWO", "1" if impl == "split_two" else "0")
    if impl == "general":
        monkeypatch.setenv("AGN_COUNTER_IMPL", "general")
    else:
        monkeypatch.delenv("AGN_COUNTER_IMPL", raising=False)
    if impl.startswith("split") and path == "host":
        pytest.skip("the host path has no hints; split covered on the device paths")
    log, req = presence_case(1000 * D + len(impl) + len(path), 260, D, 150, txid=0.3,
                             invalid=0.02, corrupt=0.03, identity=(D % 2 == 0))
    if impl.endswith("cold"):  # no SCT: the cold kernels
        req.sct = req.sct_mask = req.sct_ignore = None
    want = oracle_result(oracle_lib, log, req)
    if path == "host":
        got = eng.materialize_host(log, req, sparse=True)
    else:
        got = device_result(eng, log, req, index=(path == "device_indexed"),
                            hints={"split_ctflag": _abi.HINT_CT_FLAG,
                                   "split_mixed": _abi.HINT_MIXED}.get(impl, 0))
    bad = compare(_abi.COUNTER_PN, D, got, want, True, req.n_req)
    assert not bad, bad[:10]
    # absent LastOpCt columns are 0, as the oracle writes them (a corrupted
    # key's result is only its error)
    m = got.lastct_mask[:, 0]
    written = (got.flags & _abi.F_ERR_CORRUPTED) == 0
    for d in range(D):
        absent = (((m >> np.uint64(d)) & np.uint64(1)) == 0) & written
        assert not got.lastct[absent, d].any()


@pytest.mark.parametrize("msk", ["1", "0"])
@pytest.mark.parametrize("crdt", [_abi.SET_AW, _abi.REGISTER_MV])
@pytest.mark.parametrize("D", [2, 3, 8, 12, 16, 32, 64])
def test_tags_presence_vs_oracle(eng, oracle_lib, monkeypatch, D, crdt, msk):
    """set_aw / register_mv with presence masks: the dense passes for the keys
    whose entries share a DC set inside R (D = 2, 4, 6, 8, 16, 32, 64), the
    per-entry-mask kernel for the rest (and for every key at other widths, or
    with AGN_TAGS_MSK=0)."""
    monkeypatch.setenv("AGN_TAGS_MSK", msk)
    log, req, cap = presence_case(3000 * crdt + D, 160 if D < 32 else 90, D, 140, crdt=crdt,
                                  with_cap=True, txid=0.3, invalid=0.02, corrupt=0.03, base=0.4,
                                  multi=0.15 if crdt == _abi.SET_AW else 0.0,
                                  identity=(D % 2 == 0))
    want = oracle_result(oracle_lib, log, req, cap)
    got = eng.materialize_host(log, req, sparse=True, cap_off=cap)
    bad = compare(crdt, D, got, want, True, req.n_req)
    assert not bad, bad[:10]
    m = got.lastct_mask[:, 0]
    written = (got.flags & _abi.F_ERR_CORRUPTED) == 0
    for d in range(D):
        absent = (((m >> np.uint64(d)) & np.uint64(1)) == 0) & written
        assert not got.lastct[absent, d].any()


@pytest.mark.parametrize("D", [3, 8, 40, 64])
def test_index_masks_vs_numpy(eng, D):
    log, req, _ = random_case(77 + D, _abi.COUNTER_PN, 500, D, 90, sparse=True)
    rng = np.random.default_rng(D)
    full = (1 << D) - 1 if D < 64 else (1 << 64) - 1
    for k in range(500):
        a, b = int(log.key_off[k]), int(log.key_off[k + 1])
        if rng.random() < 0.6:
            log.oc_mask[a:b, 0] = np.uint64(int(rng.integers(1, 1 << 62)) | (1 << 63))
    dl = eng.upload_log(log)
    buf = eng.index_masks(dl)
    got = eng.download(buf, np.uint64, (500,))
    want = np.zeros(500, np.uint64)
    for k in range(500):
        a, b = int(log.key_off[k]), int(log.key_off[k + 1])
        if b == a:
            continue
        ms = log.oc_mask[a:b, 0] & np.uint64(full)
        if (ms == ms[0]).all():
            want[k] = ms[0]
    assert np.array_equal(got, want)


@pytest.mark.parametrize("impl", ["vgpr", "quad", "quad2", "split_hints"])
@pytest.mark.parametrize("D", [3, 8])
def test_full_masks_equal_dense(eng, monkeypatch, D, impl):
    """Every DC present everywhere: the masked batch equals the dense one, and
    LastOpCt's DC set is all of them (or empty when LastOpCt is ignore).
    split_hints: the early-chunk kernel with AGN_HINT_R_FULL (R masks unread)
    and AGN_HINT_CT_FLAG, over device arrays."""
    monkeypatch.delenv("AGN_COUNTER_IMPL", raising=False)
    monkeypatch.setenv("AGN_COUNTER_VARIANT", IMPLS.get(impl, "2"))
    monkeypatch.setenv("AGN_COUNTER_EARLY", "1" if impl == "split_hints" else "0")
    log, req, _ = random_case(515 + D, _abi.COUNTER_PN, 400, D, 200, sparse=True, warm=0.5,
                              txid=0.3, invalid=0.02, corrupt=0.03)
    full = np.uint64((1 << D) - 1)
    log.oc_mask[:] = full
    req.R_mask[:] = full
    req.sct_mask[:] = full
    dense = eng.materialize_host(log, req, sparse=False)
    if impl == "split_hints":
        masked = device_result(eng, log, req, index=True,
                               hints=_abi.HINT_R_FULL | _abi.HINT_CT_FLAG)
    else:
        masked = eng.materialize_host(log, req, sparse=True)
    assert not compare(_abi.COUNTER_PN, D, masked, dense, False, req.n_req)
    ign = (masked.flags & _abi.F_CT_IGNORE) != 0
    corrupt = (masked.flags & _abi.F_ERR_CORRUPTED) != 0
    ok = ~corrupt
    assert (masked.lastct_mask[ok & ~ign, 0] == full).all()
    assert (masked.lastct_mask[ok & ign, 0] == 0).all()


# ---------------------------------------------------------------- the NIF's sequence
DCAP = 8      # columns of the partition (nif_part_open's D)
JOIN = 1500   # step at which a fourth DC joins


class DictWorkload:
    """Dict clocks over interned DC columns, as nif clock_row builds them:
    DCs 0..n0-1 from the start (n0 = 3: DC 3 joins at step JOIN; n0 = DCAP:
    every column interned, full clocks throughout)."""

    def __init__(self, seed, K, n0=3, cap=DCAP):
        self.rng = np.random.default_rng(seed)
        self.cap = cap
        self.clk = np.zeros(cap, np.int64)
        self.clk[:n0] = 1000
        self.n_dc = n0
        self.K = K

    def join(self):
        self.clk[3] = 1000
        self.n_dc = 4

    def mask(self, n=None):
        return np.uint64((1 << (self.n_dc if n is None else n)) - 1)

    def op(self):
        n = self.n_dc
        c = int(self.rng.integers(0, n))
        ss = np.zeros(self.cap, np.int64)
        ss[:n] = np.maximum(self.clk[:n] - self.rng.integers(0, 40, n), 0)
        self.clk[c] += int(self.rng.integers(1, 30))
        oc = ss.copy()
        oc[c] = self.clk[c]
        return c, ss, int(self.clk[c]), oc, int(self.rng.integers(-50, 51))

    def read(self):
        lag = 400 if self.rng.random() < 0.85 else 20000
        n = self.n_dc
        if n == 4 and self.rng.random() < 0.1:
            n = 3   # a reader whose snapshot predates the new DC
        R = np.zeros(self.cap, np.int64)
        R[:n] = np.maximum(self.clk[:n] - self.rng.integers(0, lag, n), 0)
        return R, self.mask(n)


def dvc(row, n):
    return {d: int(row[d]) for d in range(n)}


# width: the partition's columns (nif_part_open's D): 8 (k_read6), 16 / 64
# (k_read6w, the fused read for wider clocks)
@pytest.mark.parametrize("width", [8, 16, 64])
@pytest.mark.parametrize("clocks", ["join", "full"])
@pytest.mark.parametrize("read6", ["1", "0"])
def test_nif_sequence_sparse_vs_dense_and_reference(eng, monkeypatch, read6, clocks, width):
    """update/2 + read/6 as nif/antidote_gpu_nif.c issues them, on a sparse
    log (presence masks; the NIF's configuration) and on a dense log: every
    read bit-identical between the two (value, NewLastOp, LastOpCt, Count,
    flags, cache status), LastOpCt's DC set inside the DCs known at the read,
    and every served value equal to the reference's ETS transcription.
    clocks = "join": 3 DCs, a fourth joining halfway (mixed keys, readers
    whose snapshot predates it); "full": every column interned from the
    start (the steady deployment: the dense routes serve every read)."""
    monkeypatch.setenv("AGN_READ6", read6)
    K, steps = 24, 3500
    w = DictWorkload(23 + width, K, n0=3 if clocks == "join" else width, cap=width)
    vn = po.MaterializerVnode()
    quirk, served, n_cmp = set(), 0, 0
    with OpLog(eng, _abi.COUNTER_PN, width, K, sparse=True) as ls, \
            OpLog(eng, _abi.COUNTER_PN, width, K, sparse=False) as ld, \
            Batcher(ls, max_batch=8, cached=True) as bs, \
            Batcher(ld, max_batch=8, cached=True) as bd:
        for s in range(steps):
            if s == JOIN and clocks == "join":
                w.join()
            key = int(w.rng.integers(0, K))
            if w.rng.random() < 0.7:
                n = w.n_dc
                c, ss, ct, oc, eff = w.op()
                pay = po.Payload(key, po.COUNTER_PN, eff, dvc(ss, n), (c, ct), s + 1)
                try:
                    vn.update(key, pay)
                except po.BadMatch:
                    quirk.add(key)
                for ol, bt, sparse in ((ls, bs, True), (ld, bd, False)):
                    if ol.gc_due(key)[0]:
                        bt.read(key, R=ss.astype(np.uint64),
                                R_mask=np.array([w.mask()]) if sparse else None, gc=True)
                    ol.append(np.array([key], np.uint64), oc.reshape(1, width).astype(np.uint64),
                              oc_mask=np.array([[w.mask()]]) if sparse else None,
                              eff=np.array([eff], np.int64), txid=np.array([s + 1], np.uint64))
                if vn.ops_cache.get(key) and any(vn.ops_cache[key][po.FIRST_OP - 1 + i] == 0
                                                 for i in range(vn.ops_cache[key][1][0])):
                    quirk.add(key)
            else:
                R, Rm = w.read()
                gs = bs.read(key, R=R.astype(np.uint64), R_mask=np.array([Rm]))
                gd = bd.read(key, R=R.astype(np.uint64))
                for f in ("status", "value", "hole", "count", "flags"):
                    assert gs[f] == gd[f], (s, key, f, gs[f], gd[f])
                if gs["status"] != _abi.SS_LOG:
                    assert np.array_equal(gs["lastct"], gd["lastct"]), (s, key)
                    assert (int(gs["lastct_mask"][0]) & ~int(w.mask())) == 0, (s, key)
                    n_cmp += 1
                if key in quirk:
                    continue
                try:
                    want = vn.read(key, po.COUNTER_PN, dvc(R, int(Rm).bit_length()), po.IGNORE)
                except NotImplementedError:
                    assert gs["status"] == _abi.SS_LOG, (s, key)
                    continue
                except po.BadMatch:
                    quirk.add(key)
                    continue
                assert gs["status"] in (_abi.SS_HIT, _abi.SS_NEW), (s, key, gs["status"])
                assert want == ("ok", gs["value"]), (s, key, want, gs["value"])
                served += 1
        lns, lls, cts = ls.key_meta()
        lnd, lld, ctd = ld.key_meta()
    assert served > 600 and n_cmp > 800, (served, n_cmp)
    assert np.array_equal(lns, lnd) and np.array_equal(lls, lld) and np.array_equal(cts, ctd)


# ---------------------------------------------------------------- full size
def entry_masks(e, D, mode, xp):
    """Deterministic per-entry presence words of a global entry index e (the
    same on the device with torch and on the host with numpy): 'full' = every
    DC, 'mixed' = one entry in 8 lacks one DC."""
    full = (1 << D) - 1
    if mode == "full":
        return e * 0 + full
    h = (e * 2654435761) & 0xFFFFFFFF
    dc = (h >> 8) % D
    one = e * 0 + 1
    drop = (h >> 29) == 0
    return xp.where(drop, full & ~(one << dc), full)


FULL_MASKED = [
    ("cfg2", dict(crdt_type=1, n_dcs=8, n_keys=10_000_000, ops_per_key=64, n_elems=0,
                  seed=20250113), "full"),
    ("cfg2", dict(crdt_type=1, n_dcs=8, n_keys=10_000_000, ops_per_key=64, n_elems=0,
                  seed=20250113), "mixed"),
    ("cfg2-warm", dict(crdt_type=1, n_dcs=8, n_keys=10_000_000, ops_per_key=64, n_elems=0,
                       seed=20250113, warm=1), "full"),
    ("cfg2-warm", dict(crdt_type=1, n_dcs=8, n_keys=10_000_000, ops_per_key=64, n_elems=0,
                       seed=20250113, warm=1), "mixed"),
    ("cfg3", dict(crdt_type=2, n_dcs=16, n_keys=1_000_000, ops_per_key=256, n_elems=32,
                  seed=20250114), "full"),
    ("cfg3", dict(crdt_type=2, n_dcs=16, n_keys=1_000_000, ops_per_key=256, n_elems=32,
                  seed=20250114), "mixed"),
]

# The forms a masked counter batch is launched in (name: hints, key_mask):
# "copy" = a key_mask buffer the context did not index (no routing by the
# log's mixed-key count), "indexed" = agn_log_index_masks' own buffer.
#   plain : k_counter_q8e, mixed keys handed on to k_counter_q8m
#   auto  : as the library routes it by itself (AGN_HINT_MIXED when more than
#           1/16 of the keys are mixed)
#   bench : AGN_HINT_CT_FLAG | AGN_HINT_R_FULL, as bench.py and the read
#           batcher pass them (LastOpCt masks over every column come back as
#           AGN_F_CT_FULL)
#   mixed : AGN_HINT_MIXED (k_counter_key, mixed keys in the same pass)
HINT_FORMS = {"plain": (0, "copy"), "auto": (0, "indexed"),
              "bench": (_abi.HINT_CT_FLAG | _abi.HINT_R_FULL, "copy"),
              "mixed": (_abi.HINT_MIXED, "copy")}


@pytest.mark.parametrize("name,spec,mode", FULL_MASKED,
                         ids=[f"{n}-{m}" for n, _, m in FULL_MASKED])
def test_full_size_masked_sampled(eng, oracle_lib, name, spec, mode):
    """BASELINE shapes with presence masks on every op clock and read (the
    NIF's partition logs, bench.py --sparse): key DC sets indexed on the
    device, every key materialized, a sample bit-exact against the oracle
    (host-generated keys with the same masks).  Counter batches run in every
    HINT_FORMS form, bench.py's hinted one included; a request flagged
    AGN_F_CT_FULL must be one whose oracle LastOpCt mask is every column."""
    import torch
    from antidote_amd.engine import free_gen_host, gen_host
    cfg = _abi.AgnGenCfg(**{"key_base": 0, "key_stride": 1, "warm": 0, **spec})
    K, D, N = cfg.n_keys, cfg.n_dcs, cfg.ops_per_key
    dl, dr = eng.gen_dev(cfg)
    E = int(dl.n_entries)
    assert E == K * N
    e = torch.arange(E, dtype=torch.int64, device="cuda")
    ocm = entry_masks(e, D, mode, torch)
    del e
    rm = torch.full((K,), (1 << D) - 1, dtype=torch.int64, device="cuda")
    dl.oc_mask, dr.R_mask = ocm.data_ptr(), rm.data_ptr()
    cap = np.arange(K + 1, dtype=np.uint64) * np.uint64(N) if cfg.crdt_type != 1 else None
    res = eng.alloc_result(K, D, sparse=True, cap_off=cap)
    kb = kcopy = None
    rng = np.random.default_rng(cfg.seed + 7)
    sample = np.sort(rng.choice(K, 48, replace=False))
    sample[0], sample[-1] = 0, K - 1
    want = {}
    for k in sample:   # the oracle on host-generated copies of the sampled keys
        c1 = _abi.AgnGenCfg(crdt_type=cfg.crdt_type, n_dcs=D, n_keys=1, ops_per_key=N,
                            n_elems=cfg.n_elems, seed=cfg.seed, key_base=int(k),
                            key_stride=1, warm=cfg.warm)
        hl, hr = gen_host(c1)
        hm = entry_masks(np.arange(int(k) * N, (int(k) + 1) * N, dtype=np.int64), D, mode,
                         np).astype(np.uint64).reshape(N, 1)
        hrm = np.full((1, 1), (1 << D) - 1, np.uint64)
        hl.oc_mask, hr.R_mask = hm.ctypes.data, hrm.ctypes.data
        capo = np.array([0, N], np.uint64) if cfg.crdt_type != 1 else None
        w = alloc_result(1, D, sparse=True, cap_off=capo)
        assert oracle_lib.oracle_materialize(C.byref(hl), C.byref(hr),
                                             C.byref(result_struct(w)), 1) == 0
        hl.oc_mask = hr.R_mask = None
        free_gen_host(hl, hr)
        want[int(k)] = w
    forms = HINT_FORMS if cfg.crdt_type == 1 else {"plain": (0, "indexed")}
    try:
        kb = eng.index_masks(dl)
        kcopy = eng.upload(eng.download(kb, np.uint64, (K,)))
        torch.cuda.synchronize()
        for form, (hints, km) in forms.items():
            dl.key_mask = (kb if km == "indexed" else kcopy).ptr
            dr.hints = hints
            eng.materialize(dl, dr, res)
            eng.sync()
            raw_flags = eng.download(res.bufs["flags"], np.uint32, (K,))
            assert not (raw_flags & (_abi.F_ERR_UNEXPECTED | _abi.F_ERR_CORRUPTED |
                                     _abi.F_ERR_CAPACITY)).any(), form
            if not hints & _abi.HINT_CT_FLAG:
                assert not (raw_flags & _abi.F_CT_FULL).any(), form
            full = eng.fetch_result(res)   # AGN_F_CT_FULL expanded to its mask word
            for k in sample:
                w = want[int(k)]
                if raw_flags[k] & _abi.F_CT_FULL:
                    assert int(w.lastct_mask[0, 0]) == (1 << D) - 1, (form, k)
                assert int(full.flags[k]) == int(w.flags[0]), (form, k)
                assert int(full.hole[k]) == int(w.hole[0]), (form, k)
                assert int(full.count[k]) == int(w.count[0]), (form, k)
                assert np.array_equal(full.lastct[k], w.lastct[0]), (form, k)
                assert np.array_equal(full.lastct_mask[k], w.lastct_mask[0]), (form, k)
                if cfg.crdt_type == 1:
                    assert int(full.value[k]) == int(w.value[0]), (form, k)
                else:
                    n, o = int(full.out_n[k]), int(full.out_off[k])
                    assert n == int(w.out_n[0]), (form, k)
                    assert np.array_equal(full.out_tag[o:o + n], w.out_tag[:n]), (form, k)
                    assert np.array_equal(full.out_tok[o:o + n], w.out_tok[:n]), (form, k)
    finally:
        dl.oc_mask = dr.R_mask = dl.key_mask = None
        eng.free_gen(dl, dr)
        for b in list(res.bufs.values()) + [x for x in (kb, kcopy) if x]:
            b.free()
        del ocm, rm
        torch.cuda.empty_cache()
