"""SURVEY.md §8(b) ownership: the engine-owned op log (agn_oplog_*), the
materializer_vnode ETS ops cache (src/materializer_vnode.erl:621-647) kept in
HBM.  A random log is appended op by op in random interleavings and batch
sizes (segments start small so they move and grow), flushed, and then:

* the op ids it assigns are the per-key counter of ets:update_counter (:630);
* agn_materialize over the flushed view (segments with key_len) is bit-exact
  with the C oracle over the same ops in CSR form;
* agn_oplog_prune leaves, per key, exactly the oracle's prune_ops output
  (snapshot_insert_gc, :513-604), and the log stays appendable after it."""
import ctypes as C

import numpy as np
import pytest

from antidote_amd import _abi
from antidote_amd.encode import (EncodedLog, alloc_result, log_struct, read_struct,
                                 result_struct, state_capacity)
from antidote_amd.engine import OpLog
from synth import compare, random_case
from test_prune import oracle_prune, thresholds

pytestmark = pytest.mark.gpu


def dl(eng, ptr, dtype, n):
    out = np.empty(n, dtype)
    if n:
        assert eng.lib.agn_memcpy_d2h(eng.ctx, out.ctypes.data, ptr, out.nbytes, None) == 0
    return out


def ops_of(log):
    """Entries grouped into ops: (key, first entry, n entries), per key oldest first."""
    ops = []
    for k in range(log.n_keys):
        a, b = int(log.key_off[k]), int(log.key_off[k + 1])
        e = a
        while e < b:
            f = e + 1
            while f < b and log.op_id[f] == log.op_id[e]:
                f += 1
            ops.append((k, e, f - e))
            e = f
    return ops


def interleave(rng, ops):
    """Random global order of the ops that keeps each key's own order."""
    by_key: dict = {}
    for op in ops:
        by_key.setdefault(op[0], []).append(op)
    seq = np.array([op[0] for op in ops], np.int64)
    rng.shuffle(seq)
    pos = {k: 0 for k in by_key}
    out = []
    for k in seq:
        out.append(by_key[k][pos[k]])
        pos[k] += 1
    return out


def append_ops(oplog, log, ops, rng, flush_p=0.5, max_batch=40):
    """Appends `ops` in random batches; returns {entry: assigned op id}."""
    tags = log.crdt_type != _abi.COUNTER_PN
    got = {}
    i = 0
    while i < len(ops):
        nb = int(rng.integers(1, max_batch + 1))
        batch = ops[i:i + nb]
        i += nb
        ent = [(k, e0 + j, j > 0) for k, e0, n in batch for j in range(n)]
        es = np.array([e for _, e, _ in ent], np.int64)
        kw = dict(oc=log.oc[es], txid=log.txid[es],
                  same_op=np.array([s for *_, s in ent], np.uint8))
        if log.oc_mask is not None:
            kw["oc_mask"] = log.oc_mask[es]
        if tags:
            lens = (log.rem_off[es + 1] - log.rem_off[es]).astype(np.int64)
            ro = np.zeros(len(es) + 1, np.uint32)
            ro[1:] = np.cumsum(lens)
            toks = [log.rem_tok[int(log.rem_off[e]):int(log.rem_off[e + 1])] for e in es]
            kw.update(tag=log.tag[es], add_tok=log.add_tok[es], rem_off=ro,
                      rem_tok=np.concatenate(toks) if toks else np.zeros(0, np.uint64))
        else:
            kw["eff"] = log.eff[es]
        ids, _ = oplog.append(np.array([k for k, _, _ in ent], np.uint64), **kw)
        for (_, e, _), op_id in zip(ent, ids):
            got[e] = int(op_id)
        if rng.random() < flush_p:
            oplog.flush()
    return got


def renumbered(log, got):
    out = EncodedLog(**{f: getattr(log, f) for f in ("crdt_type", "n_dcs", "key_off", "key_type",
                                                      "oc", "oc_mask", "txid", "eff", "tag",
                                                      "add_tok", "rem_off", "rem_tok")},
                     op_id=np.array([got[e] for e in range(log.n_entries)], np.uint32))
    return out


def expect_counter_ids(log, got, start=None):
    """Per key: ops numbered start[k]+1, +2, ... in order (ets:update_counter)."""
    for k in range(log.n_keys):
        a, b = int(log.key_off[k]), int(log.key_off[k + 1])
        nxt = 0 if start is None else int(start[k])
        for e in range(a, b):
            if e == a or log.op_id[e] != log.op_id[e - 1]:
                nxt += 1
            assert got[e] == nxt, (k, e)


def check_id_index(eng, view, K):
    """The op log keeps agn_log.key_id0 (the consecutive-op-id index) in step
    with its segments, through appends, same_op entries and prunes."""
    from test_id_index import expected_index
    assert view.key_id0
    off = dl(eng, view.key_off, np.uint64, K)
    ln = dl(eng, view.key_len, np.uint64, K)
    top = int(max((int(off[k]) + int(ln[k]) for k in range(K)), default=0))
    ids = dl(eng, view.op_id, np.uint32, top)
    assert np.array_equal(dl(eng, view.key_id0, np.uint32, K), expected_index(off, ln, ids))


def materialize_view(eng, oracle_lib, view, log, req, sparse):
    cap = state_capacity(log, req)
    dreq = eng.upload_read(req, sparse=sparse)
    dres = eng.alloc_result(req.n_req, log.n_dcs, sparse, cap_off=cap)
    eng.materialize(view, dreq, dres)
    eng.sync()
    res_g = eng.fetch_result(dres)
    res_o = alloc_result(req.n_req, log.n_dcs, sparse=sparse, cap_off=cap)
    ls, rs, os_ = log_struct(log), read_struct(req, sparse=sparse), result_struct(res_o)
    if log.oc_mask is None:
        ls.oc_mask = None
    assert oracle_lib.oracle_materialize(C.byref(ls), C.byref(rs), C.byref(os_), 4) == 0
    for d in (dreq, dres):
        for b in d.bufs.values():
            b.free()
    return compare(log.crdt_type, log.n_dcs, res_g, res_o, sparse, req.n_req)


def segments(eng, view, K, D, W, tags, sparse):
    """Downloads the view: per key a dict of its entry arrays."""
    off = dl(eng, view.key_off, np.uint64, K)
    ln = dl(eng, view.key_len, np.uint64, K)
    n = int(view.n_entries)
    arrs = {"oc": dl(eng, view.oc, np.uint64, n * D).reshape(n, D),
            "op_id": dl(eng, view.op_id, np.uint32, n), "txid": dl(eng, view.txid, np.uint64, n)}
    if sparse:
        arrs["oc_mask"] = dl(eng, view.oc_mask, np.uint64, n * W).reshape(n, W)
    if tags:
        arrs["tag"] = dl(eng, view.tag, np.uint32, n)
        arrs["add_tok"] = dl(eng, view.add_tok, np.uint64, n)
        arrs["rem_off"] = dl(eng, view.rem_off, np.uint32, n)
    else:
        arrs["eff"] = dl(eng, view.eff, np.int64, n)
    ntok = max((int(arrs["rem_off"][int(off[k]) + int(ln[k])]) for k in range(K) if ln[k]),
               default=0) if tags else 0
    tok = dl(eng, view.rem_tok, np.uint64, ntok) if ntok else np.zeros(0, np.uint64)
    out = []
    for k in range(K):
        a, b = int(off[k]), int(off[k]) + int(ln[k])
        seg = {name: v[a:b] for name, v in arrs.items() if name != "rem_off"}
        if tags:
            ro = arrs["rem_off"]
            seg["rems"] = [tok[int(ro[e]):int(ro[e + 1])].tolist() for e in range(a, b)]
        out.append(seg)
    return out


def csr_key(arrs, k, tags):
    a, b = int(arrs["key_off"][k]), int(arrs["key_off"][k + 1])
    seg = {name: v[a:b] for name, v in arrs.items()
           if v is not None and name not in ("key_off", "rem_off", "rem_tok")}
    if tags:
        ro, tok = arrs["rem_off"], arrs["rem_tok"]
        seg["rems"] = [tok[int(ro[e]):int(ro[e + 1])].tolist() for e in range(a, b)]
    return seg


CASES = [(_abi.COUNTER_PN, 8, False, 4), (_abi.COUNTER_PN, 3, True, 0),
         (_abi.COUNTER_PN, 70, True, 2), (_abi.SET_AW, 5, False, 4), (_abi.SET_AW, 16, True, 1),
         (_abi.REGISTER_MV, 8, False, 3), (_abi.REGISTER_MV, 64, True, 0)]


@pytest.mark.parametrize("crdt,D,sparse,init", CASES)
def test_oplog_append_materialize(eng, oracle_lib, crdt, D, sparse, init):
    rng = np.random.default_rng(D * 7 + crdt + 100 * init)
    log, req, _ = random_case(5 * D + crdt + init, crdt, 80, D, 70, sparse=sparse, warm=0.3,
                              txid=0.2, multi=0.2 if crdt == _abi.SET_AW else 0.0, empty=0.1)
    with OpLog(eng, crdt, D, log.n_keys, sparse=sparse, init_slots=init) as ol:
        got = append_ops(ol, log, interleave(rng, ops_of(log)), rng)
        expect_counter_ids(log, got)
        log2 = renumbered(log, got)
        view = ol.flush()
        check_id_index(eng, view, log.n_keys)
        st = ol.stats()
        assert st["entries"] == log.n_entries and st["slots"] >= log.n_entries
        assert not materialize_view(eng, oracle_lib, view, log2, req, sparse)


@pytest.fixture(params=["tail", "tail4", "tail7", "tailq2", "tailq4", "front"])
def anchor(request, monkeypatch):
    """The engine-owned log's prune kernel: k_prune_tail (kept entries compacted
    toward the end of the live range, the default; "tail4": four waves per
    block, AGN_PRUNE_WPB=4; "tail7": the compiler's register allocation,
    AGN_PRUNE_TAIL_MINW=1, instead of the default budget of 8 waves; "tailq2"
    / "tailq4": the counter form with 2 / 4 keys per wave, AGN_PRUNE_TAIL_KPW)
    or the start-anchored k_prune_inplace (AGN_PRUNE_TAIL=0)."""
    monkeypatch.setenv("AGN_PRUNE_TAIL", "0" if request.param == "front" else "1")
    monkeypatch.setenv("AGN_PRUNE_WPB", "4" if request.param == "tail4" else "1")
    monkeypatch.setenv("AGN_PRUNE_TAIL_MINW", "1" if request.param == "tail7" else "8")
    monkeypatch.setenv("AGN_PRUNE_TAIL_KPW", request.param[5:] if request.param.startswith("tailq")
                       else "1")
    return "front" if request.param == "front" else "tail"


@pytest.mark.parametrize("crdt,D,sparse,init", CASES)
def test_oplog_prune_then_append(eng, oracle_lib, anchor, crdt, D, sparse, init):
    rng = np.random.default_rng(D * 11 + crdt + init)
    tags = crdt != _abi.COUNTER_PN
    W = (D + 63) // 64
    log, req, _ = random_case(9 * D + crdt + init, crdt, 60, D, 90, sparse=sparse,
                              multi=0.2 if crdt == _abi.SET_AW else 0.0, empty=0.1)
    with OpLog(eng, crdt, D, log.n_keys, sparse=sparse, init_slots=init) as ol:
        got = append_ops(ol, log, interleave(rng, ops_of(log)), rng)
        log2 = renumbered(log, got)
        prune, thr, tm = thresholds(D + crdt + 5, log2, sparse)
        want, wflags, n_out = oracle_prune(oracle_lib, log2, prune, thr, tm)
        bp, bt = eng.upload(prune), eng.upload(thr)
        btm = eng.upload(tm) if tm is not None else None
        fl = eng.empty(4 * log.n_keys)
        ol.prune(bp.ptr, bt.ptr, btm.ptr if btm else None, fl.ptr)
        assert np.array_equal(eng.download(fl, np.uint32, (log.n_keys,)), wflags)
        assert ol.stats()["entries"] == n_out
        view = ol.flush()
        check_id_index(eng, view, log.n_keys)
        segs = segments(eng, view, log.n_keys, D, W, tags, sparse)
        for k in range(log.n_keys):
            w = csr_key(want, k, tags)
            for name, v in w.items():
                g = segs[k][name]
                if name == "rems":
                    assert g == v, (k, name)
                else:
                    assert np.array_equal(np.asarray(g), np.asarray(v)), (k, name)
        # Materialize the pruned log, then keep appending to it.
        pruned = EncodedLog(crdt_type=crdt, n_dcs=D, key_off=want["key_off"],
                            key_type=np.full(log.n_keys, crdt, np.uint8),
                            oc=want["oc"][:n_out], oc_mask=None if tm is None else
                            want["oc_mask"][:n_out], op_id=want["op_id"][:n_out],
                            txid=want["txid"][:n_out])
        if tags:
            nr = int(want["rem_off"][n_out])
            pruned.tag, pruned.add_tok = want["tag"][:n_out], want["add_tok"][:n_out]
            pruned.rem_off = want["rem_off"][:n_out + 1]
            pruned.rem_tok = want["rem_tok"][:max(nr, 1)]
        else:
            pruned.eff = want["eff"][:n_out]
        assert not materialize_view(eng, oracle_lib, view, pruned, req, sparse)

        more, req2, _ = random_case(13 * D + crdt + init, crdt, 60, D, 40, sparse=sparse,
                                    multi=0.2 if crdt == _abi.SET_AW else 0.0, empty=0.3)
        got2 = append_ops(ol, more, interleave(rng, ops_of(more)), rng)
        counters = np.zeros(log.n_keys, np.int64)
        for k in range(log.n_keys):
            a, b = int(log.key_off[k]), int(log.key_off[k + 1])
            counters[k] = max((got[e] for e in range(a, b)), default=0)
        expect_counter_ids(more, got2, counters)
        both = concat(pruned, renumbered(more, got2))
        view = ol.flush()
        check_id_index(eng, view, log.n_keys)
        assert not materialize_view(eng, oracle_lib, view, both, req2, sparse)
        for b in (bp, bt, btm, fl):
            if b is not None:
                b.free()


def pruned_log(want, n_out, crdt, D, K, sparse):
    """The oracle's prune_ops output (CSR) as an EncodedLog."""
    tags = crdt != _abi.COUNTER_PN
    out = EncodedLog(crdt_type=crdt, n_dcs=D, key_off=want["key_off"],
                     key_type=np.full(K, crdt, np.uint8), oc=want["oc"][:n_out],
                     oc_mask=want["oc_mask"][:n_out] if sparse else None,
                     op_id=want["op_id"][:n_out], txid=want["txid"][:n_out])
    if tags:
        nr = int(want["rem_off"][n_out])
        out.tag, out.add_tok = want["tag"][:n_out], want["add_tok"][:n_out]
        out.rem_off = want["rem_off"][:n_out + 1]
        out.rem_tok = want["rem_tok"][:max(nr, 1)]
    else:
        out.eff = want["eff"][:n_out]
    return out


@pytest.mark.parametrize("crdt,D,sparse", [(_abi.COUNTER_PN, 8, False), (_abi.SET_AW, 5, False),
                                           (_abi.SET_AW, 16, True), (_abi.REGISTER_MV, 64, False)])
def test_oplog_prefix_gc_cycles(eng, oracle_lib, anchor, crdt, D, sparse):
    """The common GC shape: clocks grow along each key's log, so a prune drops
    (mostly) a prefix and the tail-anchored kernel leaves the kept entries in
    place and advances the key's live range.  Six rounds of append -> prune
    (per key: nothing / a prefix / everything / not selected) -> check the
    segments, flags, id index and reads against the oracle, so live ranges
    advance, run into their segment ends, move, restart after an all-pruned
    GC, and the arenas are re-laid out."""
    rng = np.random.default_rng(D * 31 + crdt)
    K, W, tags = 48, (D + 63) // 64, crdt != _abi.COUNTER_PN
    expect = None
    counters = np.zeros(K, np.int64)
    with OpLog(eng, crdt, D, K, sparse=sparse, init_slots=4) as ol:
        for cycle in range(6):
            more, req, _ = random_case(97 * cycle + D + crdt, crdt, K, D, 24, sparse=sparse,
                                       multi=0.2 if crdt == _abi.SET_AW else 0.0, empty=0.2)
            shift = np.uint64(100_000 * (cycle + 1))     # later rounds are newer
            more.oc = more.oc + shift
            req.R = req.R + shift
            got = append_ops(ol, more, interleave(rng, ops_of(more)), rng)
            expect_counter_ids(more, got, counters)
            for k in range(K):
                a, b = int(more.key_off[k]), int(more.key_off[k + 1])
                counters[k] = max([counters[k]] + [got[e] for e in range(a, b)])
            new = renumbered(more, got)
            expect = new if expect is None else concat(expect, new)
            view = ol.flush()
            assert not materialize_view(eng, oracle_lib, view, expect, req, sparse)
            # prefix thresholds: the max OpSSCommit of the key's first `cut` ops
            thr = np.zeros((K, D), np.uint64)
            prune = (rng.random(K) < 0.85).astype(np.uint8)
            for k in range(K):
                a, b = int(expect.key_off[k]), int(expect.key_off[k + 1])
                r = rng.random()
                cut = 0 if r < 0.1 else (b - a) if r < 0.25 else int(rng.integers(0, b - a + 1))
                if cut:
                    thr[k] = expect.oc[a:a + cut].max(axis=0)
            tm = np.full((K, W), ~np.uint64(0), np.uint64) if sparse else None
            want, wflags, n_out = oracle_prune(oracle_lib, expect, prune, thr, tm)
            bp, bt = eng.upload(prune), eng.upload(thr)
            btm = eng.upload(tm) if tm is not None else None
            fl = eng.empty(4 * K)
            ol.prune(bp.ptr, bt.ptr, btm.ptr if btm else None, fl.ptr)
            assert np.array_equal(eng.download(fl, np.uint32, (K,)), wflags), cycle
            assert ol.stats()["entries"] == n_out
            view = ol.flush()
            check_id_index(eng, view, K)
            segs = segments(eng, view, K, D, W, tags, sparse)
            for k in range(K):
                for name, v in csr_key(want, k, tags).items():
                    g = segs[k][name]
                    if name == "rems":
                        assert g == v, (cycle, k, name)
                    else:
                        assert np.array_equal(np.asarray(g), np.asarray(v)), (cycle, k, name)
            expect = pruned_log(want, n_out, crdt, D, K, sparse)
            assert not materialize_view(eng, oracle_lib, view, expect, req, sparse), cycle
            for bf in (bp, bt, btm, fl):
                if bf is not None:
                    bf.free()


def long_list_log(seed, crdt, K, D, nmax):
    """A tag log whose removal lists are often long (5..150 tokens), with
    random clocks, so a prune drops entries scattered through each key and
    entries with long lists move (the kernels' entry-by-entry token copy)."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(nmax // 2, nmax + 1, K)
    key_off = np.zeros(K + 1, np.uint64)
    key_off[1:] = np.cumsum(lens)
    E = int(key_off[-1])
    rl = rng.integers(0, 3, E)
    longs = rng.random(E) < 0.3
    rl[longs] = rng.integers(5, 151, int(longs.sum()))
    rem_off = np.zeros(E + 1, np.uint32)
    rem_off[1:] = np.cumsum(rl)
    op_id = np.concatenate([np.arange(1, n + 1) for n in lens]).astype(np.uint32)
    log = EncodedLog(crdt_type=crdt, n_dcs=D, key_off=key_off,
                     key_type=np.full(K, crdt, np.uint8),
                     oc=rng.integers(1, 1000, (E, D)).astype(np.uint64), oc_mask=None,
                     op_id=op_id, txid=rng.integers(1, 6, E).astype(np.uint64))
    log.tag = rng.integers(0, 5, E).astype(np.uint32)
    log.add_tok = np.arange(1, E + 1, dtype=np.uint64) << np.uint64(8)
    log.rem_off = rem_off
    log.rem_tok = rng.integers(1, 1 << 40, max(int(rem_off[-1]), 1)).astype(np.uint64)
    return log


@pytest.mark.parametrize("crdt", [_abi.SET_AW, _abi.REGISTER_MV])
def test_oplog_prune_long_removal_lists(eng, oracle_lib, anchor, crdt):
    """Entries with removal lists longer than the kernels' register buffer
    move during an in-place prune (both anchors), twice, with appends between."""
    rng = np.random.default_rng(5 + crdt)
    K, D, W = 24, 6, 1
    log = long_list_log(41 + crdt, crdt, K, D, 70)
    _, req, _ = random_case(43 + crdt, crdt, K, D, 10)
    with OpLog(eng, crdt, D, K, init_slots=2) as ol:
        got = append_ops(ol, log, interleave(rng, ops_of(log)), rng)
        cur = renumbered(log, got)
        for rnd in range(2):
            prune, thr, _ = thresholds(61 + rnd + crdt, cur, False)
            want, wflags, n_out = oracle_prune(oracle_lib, cur, prune, thr, None)
            bp, bt, fl = eng.upload(prune), eng.upload(thr), eng.empty(4 * K)
            ol.prune(bp.ptr, bt.ptr, None, fl.ptr)
            assert np.array_equal(eng.download(fl, np.uint32, (K,)), wflags), rnd
            assert ol.stats()["entries"] == n_out
            view = ol.flush()
            check_id_index(eng, view, K)
            check_segments(eng, view, want, K, D, W, True, False)
            cur = pruned_log(want, n_out, crdt, D, K, False)
            assert not materialize_view(eng, oracle_lib, view, cur, req, False), rnd
            more = long_list_log(71 + rnd + crdt, crdt, K, D, 20)
            more.add_tok = more.add_tok + np.uint64(1 << 50)
            got2 = append_ops(ol, more, interleave(rng, ops_of(more)), rng)
            cur = concat(cur, renumbered(more, got2))
            view = ol.flush()
            assert not materialize_view(eng, oracle_lib, view, cur, req, False), rnd
            for b in (bp, bt, fl):
                b.free()


def concat(a, b):
    """Per key: a's entries then b's (both CSR)."""
    K, tags = a.n_keys, a.crdt_type != _abi.COUNTER_PN
    idx, src = [], []
    for k in range(K):
        for log, s in ((a, 0), (b, 1)):
            for e in range(int(log.key_off[k]), int(log.key_off[k + 1])):
                idx.append(e)
                src.append(s)
    lens = [int(a.key_off[k + 1] - a.key_off[k] + b.key_off[k + 1] - b.key_off[k])
            for k in range(K)]
    key_off = np.zeros(K + 1, np.uint64)
    key_off[1:] = np.cumsum(lens)
    pick = lambda name: np.array([getattr(a if s == 0 else b, name)[e]  # noqa: E731
                                  for e, s in zip(idx, src)]) if idx else \
        getattr(a, name)[:0]
    out = EncodedLog(crdt_type=a.crdt_type, n_dcs=a.n_dcs, key_off=key_off,
                     key_type=a.key_type, oc=pick("oc").reshape(-1, a.n_dcs).astype(np.uint64),
                     oc_mask=None if a.oc_mask is None else
                     pick("oc_mask").reshape(len(idx), -1).astype(np.uint64),
                     op_id=pick("op_id").astype(np.uint32), txid=pick("txid").astype(np.uint64))
    if tags:
        out.tag, out.add_tok = pick("tag").astype(np.uint32), pick("add_tok").astype(np.uint64)
        ro, toks = [0], []
        for e, s in zip(idx, src):
            lg = a if s == 0 else b
            t = lg.rem_tok[int(lg.rem_off[e]):int(lg.rem_off[e + 1])].tolist()
            toks.extend(t)
            ro.append(len(toks))
        out.rem_off = np.array(ro, np.uint32)
        out.rem_tok = np.array(toks if toks else [0], np.uint64)
    else:
        out.eff = pick("eff").astype(np.int64)
    return out


def test_oplog_gc_due_and_errors(eng):
    with OpLog(eng, _abi.COUNTER_PN, 2, 4) as ol:
        n = 120
        keys = np.zeros(n, np.uint64)
        oc = np.arange(2 * n, dtype=np.uint64).reshape(n, 2)
        ids, due = ol.append(keys, oc, eff=np.ones(n, np.int64))
        assert ids.tolist() == list(range(1, n + 1))
        # op_insert_gc's trigger (:635): Length >= ListLen or NewId rem 50 == 0;
        # the segment doubles 50 -> 100 -> 200 instead of forcing the GC.
        assert np.flatnonzero(due).tolist() == [49, 50, 99, 100]
        before = ol.stats()
        with pytest.raises(Exception):
            ol.append(np.array([1, 9], np.uint64), oc[:2], eff=np.ones(2, np.int64))
        with pytest.raises(Exception):
            ol.append(np.array([1], np.uint64), oc[:1], eff=np.ones(1, np.int64),
                      same_op=np.ones(1, np.uint8))
        assert ol.stats() == before  # rejected batches leave no trace
        ids, _ = ol.append(np.array([1, 1, 0], np.uint64), oc[:3], eff=np.ones(3, np.int64),
                           same_op=np.array([0, 1, 0], np.uint8))
        assert ids.tolist() == [1, 1, 121]
        view = ol.flush()
        assert dl(eng, view.key_len, np.uint64, 4).tolist() == [121, 2, 0, 0]


def new_list_len(new_length, list_len):
    """snapshot_insert_gc's NewListLen (src/materializer_vnode.erl:540-558)."""
    if new_length > list_len - _abi.RESIZE_THRESHOLD:
        return list_len * 2
    half = list_len // 2
    if half <= _abi.OPS_THRESHOLD:
        return list_len
    return half if half - _abi.RESIZE_THRESHOLD > new_length else list_len


def expected_meta(before, prune, kept):
    """Per key {Length, ListLen, OpId} after a prune: selected keys get the
    kept length and the resized ListLen (prune_ops' NewLength is 1 when no op
    survives, :580-583), the others and every op counter are unchanged."""
    ln, ll, ct = (x.copy() for x in before)
    for k in range(len(ln)):
        if prune[k]:
            ln[k] = kept[k]
            if ll[k]:
                ll[k] = max(new_list_len(max(int(kept[k]), 1), int(ll[k])), int(kept[k]))
    return ln, ll, ct


def check_segments(eng, view, want, K, D, W, tags, sparse):
    segs = segments(eng, view, K, D, W, tags, sparse)
    for k in range(K):
        w = csr_key(want, k, tags)
        for name, v in w.items():
            g = segs[k][name]
            if name == "rems":
                assert g == v, (k, name)
            else:
                assert np.array_equal(np.asarray(g), np.asarray(v)), (k, name)


@pytest.mark.parametrize("crdt,D,sparse", [(_abi.COUNTER_PN, 8, False), (_abi.SET_AW, 12, True),
                                           (_abi.REGISTER_MV, 3, False)])
def test_oplog_resize_policy_and_relayout(eng, oracle_lib, monkeypatch, crdt, D, sparse):
    """The ETS resize policy after a prune (ListLen doubles / halves / stays,
    per key, against the reference's NewListLen), then the relayout of the
    fragmented arenas: refused once by a forced allocation failure (the log
    must come through unchanged and correct), done on the next prune; the
    log stays bit-exact and appendable throughout."""
    rng = np.random.default_rng(77 + D + crdt)
    tags = crdt != _abi.COUNTER_PN
    W = (D + 63) // 64
    K = 120
    log, req, _ = random_case(31 * D + crdt, crdt, K, D, 260, sparse=sparse,
                              multi=0.2 if crdt == _abi.SET_AW else 0.0, empty=0.05)
    with OpLog(eng, crdt, D, K, sparse=sparse, init_slots=1) as ol:
        got = append_ops(ol, log, interleave(rng, ops_of(log)), rng, flush_p=0.2)
        log2 = renumbered(log, got)
        before = ol.key_meta()
        prune, thr, tm = thresholds(3 * D + crdt, log2, sparse)
        want, wflags, n_out = oracle_prune(oracle_lib, log2, prune, thr, tm)
        kept = np.diff(want["key_off"]).astype(np.int64)
        bp, bt = eng.upload(prune), eng.upload(thr)
        btm = eng.upload(tm) if tm is not None else None
        fl = eng.empty(4 * K)
        ol.prune(bp.ptr, bt.ptr, btm.ptr if btm else None, fl.ptr)
        after = ol.key_meta()
        exp = expected_meta(before, prune, kept)
        for name, g, w in zip(("Length", "ListLen", "OpId"), after, exp):
            assert np.array_equal(g, w), (name, np.flatnonzero(g != w)[:5])
        assert (after[1] != before[1]).any()
        assert np.array_equal(eng.download(fl, np.uint32, (K,)), wflags)
        slots0 = ol.stats()["slots"]
        # a prune selecting nothing: the relayout is wanted, its first
        # allocation fails -> skipped, the log is untouched
        none = eng.upload(np.zeros(K, np.uint8))
        monkeypatch.setenv("AGN_TEST_POOL_FAIL", "1")
        ol.prune(none.ptr, bt.ptr, btm.ptr if btm else None)
        monkeypatch.delenv("AGN_TEST_POOL_FAIL")
        assert ol.stats()["slots"] == slots0
        view = ol.flush()
        check_segments(eng, view, want, K, D, W, tags, sparse)
        # the next prune re-lays the arenas out
        ol.prune(none.ptr, bt.ptr, btm.ptr if btm else None)
        assert ol.stats()["slots"] < slots0 // 2 + 1, (ol.stats()["slots"], slots0)
        assert all(np.array_equal(a, b) for a, b in zip(ol.key_meta(), after))
        view = ol.flush()
        check_id_index(eng, view, K)
        check_segments(eng, view, want, K, D, W, tags, sparse)
        # appends past the shrunk ListLens, then a full materialize
        more, req2, _ = random_case(17 * D + crdt, crdt, K, D, 80, sparse=sparse,
                                    multi=0.2 if crdt == _abi.SET_AW else 0.0, empty=0.2)
        got2 = append_ops(ol, more, interleave(rng, ops_of(more)), rng)
        pruned = EncodedLog(crdt_type=crdt, n_dcs=D, key_off=want["key_off"],
                            key_type=np.full(K, crdt, np.uint8), oc=want["oc"][:n_out],
                            oc_mask=None if tm is None else want["oc_mask"][:n_out],
                            op_id=want["op_id"][:n_out], txid=want["txid"][:n_out])
        if tags:
            nr = int(want["rem_off"][n_out])
            pruned.tag, pruned.add_tok = want["tag"][:n_out], want["add_tok"][:n_out]
            pruned.rem_off = want["rem_off"][:n_out + 1]
            pruned.rem_tok = want["rem_tok"][:max(nr, 1)]
        else:
            pruned.eff = want["eff"][:n_out]
        both = concat(pruned, renumbered(more, got2))
        view = ol.flush()
        check_id_index(eng, view, K)
        assert not materialize_view(eng, oracle_lib, view, both, req2, sparse)
        for b in (bp, bt, btm, fl, none):
            if b is not None:
                b.free()


def test_oplog_resize_policy_directions(eng):
    """Deterministic NewListLen cases (OPS_THRESHOLD = 50 slots at first):
    key 0: 48 ops, nothing pruned -> 48 > 50 - 5: ListLen doubles to 100;
    key 1: 200 ops (ListLen 50 -> 100 -> 200), 10 kept -> halves to 100;
    key 2: 60 ops (ListLen 100), 30 kept -> half = 50 <= OPS_THRESHOLD: stays;
    key 3: 3 ops, all pruned -> NewLength 1: 50 stays (and AGN_GC_ALL_PRUNED);
    key 4: never written -> ListLen 0 stays 0."""
    D, K = 2, 5
    lens = [48, 200, 60, 3, 0]
    kept = [48, 10, 30, 0, 0]
    with OpLog(eng, _abi.COUNTER_PN, D, K) as ol:
        keys = np.concatenate([np.full(n, k, np.uint64) for k, n in enumerate(lens)])
        pos = np.concatenate([np.arange(n) for n in lens]).astype(np.uint64)
        oc = np.stack([pos + 1, pos + 1], axis=1).astype(np.uint64)   # op i: clock i+1
        ol.append(keys, oc, eff=np.ones(len(keys), np.int64))
        ln, ll, ct = ol.key_meta()
        assert ln.tolist() == lens and ll.tolist() == [50, 200, 100, 50, 0]
        # threshold t covers ops with clock <= t: keep the newest kept[k] ops
        thr = np.array([[n - m, n - m] for n, m in zip(lens, kept)], np.uint64)
        bt, bp, fl = eng.upload(thr), eng.upload(np.ones(K, np.uint8)), eng.empty(4 * K)
        ol.prune(bp.ptr, bt.ptr, None, fl.ptr)
        ln, ll, ct2 = ol.key_meta()
        assert ln.tolist() == kept
        assert ll.tolist() == [100, 100, 100, 50, 0]
        assert ct2.tolist() == ct.tolist()
        assert eng.download(fl, np.uint32, (K,)).tolist() == [0, 0, 0, _abi.GC_ALL_PRUNED,
                                                              _abi.GC_ALL_PRUNED]
        # op_insert_gc's trigger now counts against the new ListLen (:635)
        _, due = ol.append(np.array([1] * 91, np.uint64), np.full((91, D), 10 ** 6, np.uint64),
                           eff=np.ones(91, np.int64))
        # ids 201..291: id 250 (NewId rem 50 == 0) and the 91st (Length 100 >= ListLen 100)
        assert np.flatnonzero(due).tolist() == [49, 90]
        for b in (bt, bp, fl):
            b.free()
