"""GC of the op log — materializer_vnode
snapshot_insert_gc -> prune_ops/check_filter (src/materializer_vnode.erl:513-604).

The C oracle's SoA compaction is checked against the literal ETS-tuple
transcription in oracle/py_oracle.py (MaterializerVnode.prune_ops, including
the all-pruned quirk of :580-583), and the GPU's three-pass compaction
(agn_prune_ops) against the C oracle on every output array."""
import ctypes as C

import numpy as np
import pytest

from antidote_amd import _abi
from antidote_amd.encode import log_struct
from oracle import py_oracle as po
from synth import random_case
from test_oracle_crosscheck import TYPES, key_ops, to_dict


def thresholds(seed, log, sparse):
    """Per key: max OpSSCommit of a random prefix of its ops, jittered; some
    keys get a threshold covering everything (the all-pruned case)."""
    rng = np.random.default_rng(seed)
    K, D = log.n_keys, log.n_dcs
    W = (D + 63) // 64
    thr = np.zeros((K, D), np.uint64)
    for k in range(K):
        a, b = int(log.key_off[k]), int(log.key_off[k + 1])
        if b == a:
            thr[k] = rng.integers(0, 100, D)
            continue
        cut = int(rng.integers(0, b - a + 1))
        if rng.random() < 0.1:
            cut = b - a
        base = log.oc[a:a + cut].max(axis=0) if cut else log.oc[a].astype(np.int64) - 100
        thr[k] = np.maximum(base.astype(np.int64) + rng.integers(-3, 4, D), 0)
        if rng.random() < 0.1:
            thr[k] = np.iinfo(np.uint64).max // 2
    tm = None
    if sparse:
        tm = np.zeros((K, W), np.uint64)
        pres = rng.random((K, D)) >= 0.1
        for d in range(D):
            tm[:, d >> 6] |= pres[:, d].astype(np.uint64) << np.uint64(d & 63)
    prune = (rng.random(K) < 0.8).astype(np.uint8)
    return prune, thr, tm


def host_out_like(log):
    """numpy arrays sized like the input, zero-filled (agn_prune_ops contract)."""
    out = {}
    for name in ("key_off", "oc", "oc_mask", "op_id", "txid", "eff", "tag", "add_tok",
                 "rem_off", "rem_tok"):
        a = getattr(log, name)
        out[name] = None if a is None else np.zeros_like(a)
    return out


def out_struct(log, arrs):
    s = _abi.AgnLog()
    s.crdt_type, s.n_dcs, s.n_keys = log.crdt_type, log.n_dcs, log.n_keys
    for name, a in arrs.items():
        setattr(s, name, None if a is None or a.size == 0 else a.ctypes.data)
    return s


def oracle_prune(lib, log, prune, thr, tm):
    arrs = host_out_like(log)
    ls = log_struct(log)
    if log.oc_mask is None:
        ls.oc_mask = None
    os_ = out_struct(log, arrs)
    flags = np.zeros(log.n_keys, np.uint32)
    p = lambda a: None if a is None else a.ctypes.data  # noqa: E731
    assert lib.oracle_prune_ops(C.byref(ls), p(prune), p(thr), p(tm), C.byref(os_),
                                p(flags)) == 0
    return arrs, flags, int(os_.n_entries)


CASES = [(_abi.COUNTER_PN, 3, False), (_abi.COUNTER_PN, 8, True), (_abi.COUNTER_PN, 16, False),
         (_abi.SET_AW, 5, False), (_abi.SET_AW, 16, True), (_abi.REGISTER_MV, 64, False),
         (_abi.REGISTER_MV, 2, True)]


@pytest.mark.parametrize("crdt,D,sparse", CASES)
def test_oracle_prune_vs_ets_transcription(oracle_lib, crdt, D, sparse):
    log, _req, _ = random_case(31 * D + crdt + sparse, crdt, 60, D, 90, sparse=sparse,
                               multi=0.2 if crdt == _abi.SET_AW else 0.0, empty=0.1)
    prune, thr, tm = thresholds(D + crdt, log, sparse)
    arrs, flags, n_out = oracle_prune(oracle_lib, log, prune, thr, tm)
    assert n_out == int(arrs["key_off"][-1])
    W = (D + 63) // 64
    for k in range(log.n_keys):
        ops = key_ops(log, k, TYPES[crdt])[::-1]  # oldest first: the tuple order
        got_ids = []
        for e in range(int(arrs["key_off"][k]), int(arrs["key_off"][k + 1])):
            if not got_ids or got_ids[-1] != int(arrs["op_id"][e]):
                got_ids.append(int(arrs["op_id"][e]))
        if not prune[k]:
            assert got_ids == [i for i, _ in ops]
            continue
        tup = po.EtsTuple(["k", (len(ops), len(ops) + 5), 0] + list(ops) + [0] * 6)
        threshold = to_dict(thr[k], None if tm is None else tm[k], D)
        size, kept = po.MaterializerVnode.prune_ops(len(ops), tup, threshold)
        if all(el == 0 for _slot, el in kept):  # :580-583 quirk (also for 0 ops)
            assert flags[k] == _abi.GC_ALL_PRUNED and got_ids == []
        else:
            assert flags[k] == 0
            assert got_ids == [el[0] for _slot, el in kept]
            assert size == len(got_ids)
    assert flags.any() and (flags == 0).any()
    assert 0 < n_out < log.n_entries
    _ = W


@pytest.mark.gpu
@pytest.mark.parametrize("crdt,D,sparse", CASES + [(_abi.COUNTER_PN, 256, True),
                                                   (_abi.SET_AW, 100, False)])
def test_prune_gpu_vs_oracle(eng, oracle_lib, crdt, D, sparse):
    log, _req, _ = random_case(77 * D + crdt + sparse, crdt, 200, D, 150 if D <= 16 else 60,
                               sparse=sparse, multi=0.2 if crdt == _abi.SET_AW else 0.0,
                               empty=0.1, txid=0.0)
    prune, thr, tm = thresholds(D * 3 + crdt, log, sparse)
    want, wflags, n_out = oracle_prune(oracle_lib, log, prune, thr, tm)
    dlog = eng.upload_log(log)
    if log.oc_mask is None:
        dlog.struct.oc_mask = None
    dout = eng.alloc_log_like(log)
    bp, bt = eng.upload(prune), eng.upload(thr)
    btm = eng.upload(tm) if tm is not None else None
    fl, tot = eng.empty(4 * log.n_keys), eng.empty(16)
    eng.prune_ops(dlog, bp.ptr, bt.ptr, btm.ptr if btm else None, dout, fl.ptr, tot.ptr)
    eng.sync()
    totals = eng.download(tot, np.uint64, (2,))
    assert int(totals[0]) == n_out
    assert np.array_equal(eng.download(fl, np.uint32, (log.n_keys,)), wflags)
    for name, (dt, shape) in dout.shapes.items():
        got = eng.download(dout.bufs[name], dt, shape)
        w = want[name]
        if name == "key_off":
            assert np.array_equal(got, w), name
            continue
        if name == "rem_off":
            assert np.array_equal(got[:n_out + 1], w[:n_out + 1]), name
            continue
        if name == "rem_tok":
            nr = int(totals[1])
            assert nr == int(want["rem_off"][n_out])
            assert np.array_equal(got[:nr], w[:nr]), name
            continue
        assert np.array_equal(got[:n_out], w[:n_out]), name


@pytest.mark.gpu
@pytest.mark.parametrize("crdt,D,sparse", CASES + [(_abi.COUNTER_PN, 256, True),
                                                   (_abi.SET_AW, 100, False),
                                                   (_abi.COUNTER_PN, 8, False)])
@pytest.mark.parametrize("ct", ["0", "1", "pf0", "pf1", "pf2", "pf3", "mw8"])
def test_prune_segmented_gpu_vs_oracle(eng, oracle_lib, monkeypatch, crdt, D, sparse, ct):
    """agn_prune_ops with out.key_len: the one-pass segmented form -- every
    key's kept entries at its input segment start, bit-exact with the
    oracle's CSR output key by key, unselected keys copied, plus the
    consecutive-id index.  ct = "1": contiguous row loads (AGN_PRUNE_CT);
    "pf1" / "pf2": the next iteration's rows prefetched (AGN_PRUNE_PF; "pf3"
    with the next fields predicted; "pf0" none, the default being 1 for
    set/register); "mw8":
    the register budget of 8 waves per SIMD (AGN_PRUNE_MINW, spills)."""
    from test_id_index import expected_index
    monkeypatch.setenv("AGN_PRUNE_CT", ct if ct in ("0", "1") else "0")
    if ct.startswith("pf"):
        monkeypatch.setenv("AGN_PRUNE_PF", ct[2:])
    else:
        monkeypatch.delenv("AGN_PRUNE_PF", raising=False)
    monkeypatch.setenv("AGN_PRUNE_MINW", ct[2:] if ct.startswith("mw") else "1")
    log, _req, _ = random_case(91 * D + crdt + sparse, crdt, 200, D, 150 if D <= 16 else 60,
                               sparse=sparse, multi=0.2 if crdt == _abi.SET_AW else 0.0,
                               empty=0.1, txid=0.3)
    prune, thr, tm = thresholds(D * 5 + crdt, log, sparse)
    want, wflags, n_out = oracle_prune(oracle_lib, log, prune, thr, tm)
    K = log.n_keys
    dlog = eng.upload_log(log)
    if log.oc_mask is None:
        dlog.struct.oc_mask = None
    dout = eng.alloc_log_like(log)
    kl, kid = eng.empty(8 * K), eng.empty(4 * K)
    dout.struct.key_len, dout.struct.key_id0 = kl.ptr, kid.ptr
    bp, bt = eng.upload(prune), eng.upload(thr)
    btm = eng.upload(tm) if tm is not None else None
    fl, tot = eng.empty(4 * K), eng.empty(16)
    eng.prune_ops(dlog, bp.ptr, bt.ptr, btm.ptr if btm else None, dout, fl.ptr, tot.ptr)
    eng.sync()
    totals = eng.download(tot, np.uint64, (2,))
    assert int(totals[0]) == n_out
    assert int(totals[1]) == int(want["rem_off"][n_out]) if log.rem_off is not None else True
    assert np.array_equal(eng.download(fl, np.uint32, (K,)), wflags)
    starts = eng.download(dout.bufs["key_off"], np.uint64, (K + 1,))[:K]
    lens = eng.download(kl, np.uint64, (K,))
    assert np.array_equal(starts, log.key_off[:K])
    assert np.array_equal(lens, np.diff(want["key_off"]))
    got = {n: eng.download(dout.bufs[n], *dout.shapes[n]) for n in dout.shapes}
    for k in range(K):
        a, b = int(starts[k]), int(starts[k]) + int(lens[k])
        wa, wb = int(want["key_off"][k]), int(want["key_off"][k + 1])
        for name in ("oc", "oc_mask", "op_id", "txid", "eff", "tag", "add_tok"):
            if name in got:
                assert np.array_equal(got[name][a:b], want[name][wa:wb]), (k, name)
        if log.rem_off is not None:
            ro, wro = got["rem_off"], want["rem_off"]
            for e, we in zip(range(a, b), range(wa, wb)):
                g = got["rem_tok"][int(ro[e]):int(ro[e + 1])]
                w = want["rem_tok"][int(wro[we]):int(wro[we + 1])]
                assert np.array_equal(g, w), (k, e)
    ids = got["op_id"]
    assert np.array_equal(eng.download(kid, np.uint32, (K,)), expected_index(starts, lens, ids))
