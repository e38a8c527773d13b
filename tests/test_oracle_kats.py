"""Pin both oracles (oracle/py_oracle.py and oracle/oracle.c) against the
reference's own known answers (tests/golden/kats.json, transcribed from the
EUnit / common_test suites by tests/golden/make_kats.py)."""
import ctypes as C

import numpy as np
import pytest

from antidote_amd import _abi
from kat_util import (TYPES, OneKeyRun, kats, oracle_fn, py_ops, system_seq_log, system_txn_log,
                      to_payload,
                      to_vc)
from oracle import py_oracle as po

MAT = kats({"materialize", "materialize_chain"})


def _resp(ops, sct, base):
    return po.SnapshotGetResponse(ops, len(ops), po.MaterializedSnapshot(base[0], base[1]),
                                  sct, True)


def py_materialize_case(c):
    typ = TYPES[c["type"]]
    ops = py_ops(c)
    if c["kind"] == "materialize_chain":
        f = c["first"]
        r1 = po.materialize(typ, po.IGNORE, to_vc(f["R"]), _resp(ops, to_vc(f["sct"]), f["base"]))
        _, v1, hole1, ct1, _, _ = r1
        return po.materialize(typ, po.IGNORE, to_vc(c["R"]), _resp(ops, ct1, [hole1, v1]))
    return po.materialize(typ, po.IGNORE, to_vc(c["R"]), _resp(ops, to_vc(c["sct"]), c["base"]))


def check_expect(r, exp):
    assert r[0] == "ok", r
    _, value, hole, ct, _newss, _count = r
    if "value" in exp:
        assert value == exp["value"]
    if "hole" in exp:
        assert hole == exp["hole"]
    if "ct" in exp:
        assert ct == (po.IGNORE if exp["ct"] is None else to_vc(exp["ct"]))


@pytest.mark.parametrize("c", MAT, ids=[c["name"] for c in MAT])
def test_py_oracle_materialize(c):
    check_expect(py_materialize_case(c), c["expect"])


def c_materialize_case(fn, c):
    """fn(log_struct, read_struct, result_struct) -> rc (C oracle or engine)."""
    ops = py_ops(c)
    clocks = [p.snapshot_time for _, p in ops] + [to_vc(c["R"])]
    n_dcs = max(2, len({d for ck in clocks for d in ck} | {p.commit_time[0] for _, p in ops}))
    run = OneKeyRun(c["type"], ops, n_dcs)
    if c["kind"] == "materialize_chain":
        f = c["first"]
        run.add_read(to_vc(f["R"]), to_vc(f["sct"]), base=f["base"][1])
        _, res = run.run(fn)
        _, v1, hole1, ct1, _, _ = run.decode(res, 0)
        run2 = OneKeyRun(c["type"], ops, n_dcs)
        run2.add_read(to_vc(c["R"]), ct1, base=v1)
        _, res2 = run2.run(fn)
        return run2.decode(res2, 0)
    run.add_read(to_vc(c["R"]), to_vc(c["sct"]), base=c["base"][1])
    _, res = run.run(fn)
    return run.decode(res, 0)


@pytest.mark.parametrize("c", MAT, ids=[c["name"] for c in MAT])
def test_c_oracle_materialize(oracle_lib, c):
    r = c_materialize_case(oracle_fn(oracle_lib), c)
    check_expect(r, c["expect"])
    # the two restatements agree on every field, asserted or not
    py = py_materialize_case(c)
    assert r == py


EAGER = kats({"eager"})


@pytest.mark.parametrize("c", EAGER, ids=[c["name"] for c in EAGER])
def test_eager(oracle_lib, c):
    typ = TYPES[c["type"]]
    effs = [tuple(e.values()) if isinstance(e, dict) else e for e in c["effects"]]
    r = po.materialize_eager(typ, po.crdt_new(typ), effs)
    exp = c["expect"]
    if "error" in exp:
        assert r == ("error", ("unexpected_operation", effs[exp["op_index"]], typ))
    else:
        assert r == exp["value"]
    # C oracle: the same effects as a single-DC log, all included
    ops = [(i + 1, po.Payload("k", typ, e, {1: 10 * i}, (1, 10 * i + 5), i + 1))
           for i, e in enumerate(effs)][::-1]
    run = OneKeyRun(c["type"], ops, 1)
    run.add_read({1: 10 ** 9})
    _, res = run.run(oracle_fn(oracle_lib))
    cr = run.decode(res, 0)
    if "error" in exp:
        assert cr[0] == "error" and cr[1][0] == "unexpected_operation"
        assert cr[1][1] == effs[exp["op_index"]]
    else:
        assert cr[1] == exp["value"] and cr[5] == len(effs)


ISOP = kats({"is_op_in_snapshot"})


@pytest.mark.parametrize("c", ISOP, ids=[c["name"] for c in ISOP])
def test_is_op_in_snapshot(oracle_lib, c):
    p = to_payload(c["op"], po.COUNTER_PN)
    got = po.is_op_in_snapshot(c["txid"], p, p.commit_time, p.snapshot_time,
                               to_vc(c["snapshot"]), po.IGNORE, po.IGNORE)
    e = c["expect"]
    assert got == (e["incl"], e["in_prev"], to_vc(e["time"]))
    # C oracle: one-op log, effect replaced by an integer
    q = po.Payload("k", po.COUNTER_PN, 2, p.snapshot_time, p.commit_time, p.txid)
    run = OneKeyRun("counter_pn", [(1, q)], 1)
    run.add_read(to_vc(c["snapshot"]), txid=c["txid"])
    _, res = run.run(oracle_fn(oracle_lib))
    _, _, _, ct, newss, count = run.decode(res, 0)
    assert newss == e["incl"] and count == int(e["incl"])
    assert ct == to_vc(e["time"])


BEL = kats({"belongs_to_snapshot_op"})


@pytest.mark.parametrize("c", BEL, ids=[c["name"] for c in BEL])
def test_belongs_to_snapshot_op(oracle_lib, c):
    sct, (dc, t), ss = to_vc(c["sct"]), c["dc_ct"], to_vc(c["op_ss"])
    assert po.belongs_to_snapshot_op(sct, (dc, t), ss) == c["expect"]["result"]
    oc = dict(ss)
    oc[dc] = t
    dcs = sorted(set(oc) | set(sct))
    a = np.array([oc.get(d, 0) for d in dcs], np.uint64)
    b = np.array([sct.get(d, 0) for d in dcs], np.uint64)
    am = np.array([sum(1 << i for i, d in enumerate(dcs) if d in oc)], np.uint64)
    bm = np.array([sum(1 << i for i, d in enumerate(dcs) if d in sct)], np.uint64)
    le = oracle_lib.oracle_vc_le(len(dcs), a.ctypes.data, am.ctypes.data, b.ctypes.data,
                                 bm.ctypes.data)
    assert (not le) == c["expect"]["result"]


VNODE = kats({"vnode"})


@pytest.mark.parametrize("c", VNODE, ids=[c["name"] for c in VNODE])
def test_py_oracle_vnode(c):
    typ = TYPES[c["type"]]
    v = po.MaterializerVnode()
    for st in c["steps"]:
        if st[0] == "update":
            _, key, p = st
            v.update(key, to_payload(p, typ))
        else:
            _, key, r, gc, want = st
            ok, val = v.internal_read(key, typ, to_vc(r), po.IGNORE, gc)
            assert ok == "ok" and po.crdt_value(typ, val) == want, (st, val)


ORD = kats({"orddict_insert_then", "orddict_insert_bigger", "orddict_filter_gt_new",
            "orddict_conc"})


def _ent(e):
    return None if e is None else (to_vc(e[0]), e[1])


@pytest.mark.parametrize("c", ORD, ids=[c["name"] for c in ORD])
def test_vector_orddict(oracle_lib, c):
    k = c["kind"]
    if k == "orddict_insert_then":
        d = po.VectorOrddict()
        for clock, val in c["inserts"]:
            d = d.insert(to_vc(clock), val)
        for chk in c["checks"]:
            if chk[0] == "get_smaller_from_id":
                target = po.VectorOrddict() if len(chk) > 3 else d
                dc, t = chk[1]
                assert target.get_smaller_from_id(dc, t) == _ent(chk[2])
            else:
                found, first = d.get_smaller(to_vc(chk[1]))
                assert (found, first) == (_ent(chk[2][0]), chk[2][1])
                # C oracle select_base on the same list
                dcs = ["dc1", "dc2"]
                clocks = np.array([[cl.get(x, 0) for x in dcs] for cl, _ in d.lst], np.uint64)
                cm = np.array([[sum(1 << i for i, x in enumerate(dcs) if x in cl)]
                               for cl, _ in d.lst], np.uint64)
                rv = to_vc(chk[1])
                R = np.array([[rv.get(x, 0) for x in dcs]], np.uint64)
                Rm = np.array([[sum(1 << i for i, x in enumerate(dcs) if x in rv)]], np.uint64)
                off = np.array([0, len(d.lst)], np.uint64)
                idx = np.zeros(1, np.int32)
                isf = np.zeros(1, np.uint8)
                oracle_lib.oracle_select_base(2, 1, off.ctypes.data, clocks.ctypes.data,
                                              cm.ctypes.data, R.ctypes.data, Rm.ctypes.data,
                                              idx.ctypes.data, isf.ctypes.data)
                want_idx = -1 if found is None else [x[1] for x in d.lst].index(found[1])
                assert (int(idx[0]), bool(isf[0])) == (want_idx, first)
    elif k == "orddict_insert_bigger":
        d = po.VectorOrddict()
        for clock, val, size in c["steps"]:
            d = d.insert_bigger(to_vc(clock), val)
            assert d.size() == size
    elif k == "orddict_filter_gt_new":
        d = po.VectorOrddict([_ent(e) for e in c["entries"]])
        res = d.filter(lambda x: po.vc_gt(x[0], {}))
        assert res.lst == [_ent(e) for e in c["expect"]]
    else:
        d = po.VectorOrddict([_ent(e) for e in c["entries"]])
        for clock, want in c["checks"]:
            assert d.is_concurrent_with_any(to_vc(clock)) == want


GST = kats({"gst"})


@pytest.mark.parametrize("c", GST, ids=[c["name"] for c in GST])
def test_gst_get_min_time(oracle_lib, c):
    parts = {p: (po.UNDEFINED if v == "undefined" else to_vc(v)) for p, v in c["parts"].items()}
    want = to_vc(c["expect"])
    assert po.get_min_time(parts) == want
    dcs = sorted({d for v in parts.values() if v != po.UNDEFINED for d in v}) or ["dc1"]
    D, P = len(dcs), len(parts)
    clocks = np.full((P, D), _abi.U64_MAX, np.uint64)
    defined = np.ones(P, np.uint8)
    for i, v in enumerate(parts.values()):
        if v == po.UNDEFINED:
            defined[i] = 0
        else:
            for j, d in enumerate(dcs):
                if d in v:
                    clocks[i, j] = v[d]
    out = np.zeros(D + 1, np.uint64)
    oracle_lib.oracle_gst_min(D, P, 1, clocks.ctypes.data, defined.ctypes.data,
                              out.ctypes.data, 1)
    got = {d: int(out[j]) for j, d in enumerate(dcs) if int(out[j]) != _abi.U64_MAX}
    assert got == want


def test_update_stable(oracle_lib):
    last = {"dc1": 5, "dc2": 9}
    changed, acc = po.update_stable(last, {"dc1": 7, "dc2": 3, "dc3": 1})
    assert changed and acc == {"dc1": 7, "dc2": 9, "dc3": 1}
    changed, acc = po.update_stable(acc, {"dc2": 1})
    assert not changed
    L = np.array([5, 9, _abi.U64_MAX], np.uint64)
    N = np.array([7, 3, 1], np.uint64)
    ch = C.c_int(0)
    oracle_lib.oracle_update_stable(3, L.ctypes.data, N.ctypes.data, C.byref(ch))
    assert ch.value == 1 and L.tolist() == [7, 9, 1]


SYS = kats({"system_seq"})


@pytest.mark.parametrize("c", SYS, ids=[c["name"] for c in SYS])
def test_system_seq(oracle_lib, c):
    typ = TYPES[c["type"]]
    ops, reads, _ = system_seq_log(c)
    exp = c["expect_after"]
    checks = (list(enumerate(exp)) if isinstance(exp, list)
              else [(int(k) - 1, v) for k, v in exp.items()])
    for i, want in checks:
        r = po.materialize(typ, po.IGNORE, reads[i],
                           _resp(ops, po.IGNORE, [0, po.crdt_new(typ)]))
        assert po.crdt_value(typ, r[1]) == want
        if "expect_state_tokens_per_elem" in c:
            assert all(len(toks) == 1 for _, toks in r[1])
        run = OneKeyRun(c["type"], ops, 1)
        run.add_read(reads[i])
        _, res = run.run(oracle_fn(oracle_lib))
        cr = run.decode(res, 0)
        assert cr == r


TXN = kats({"system_txn"})


def system_txn_check(c, materialize_fn):
    """Every read of a system_txn KAT: the dict restatement must give the
    value the reference asserts, and the SoA path through materialize_fn (C
    oracle or HIP engine) must give the restatement's full result tuple."""
    typ = TYPES[c["type"]]
    logs, reads = system_txn_log(c)
    n_dcs = len({t["dc"] for t in c["txns"]})
    for key, R, want in reads:
        ops = logs.get(key, [])
        r = po.materialize(typ, po.IGNORE, R, _resp(ops, po.IGNORE, [0, po.crdt_new(typ)]))
        assert r[0] == "ok" and po.crdt_value(typ, r[1]) == want, (key, r)
        run = OneKeyRun(c["type"], ops, n_dcs)
        run.add_read(R)
        _, res = run.run(materialize_fn)
        got = run.decode(res, 0)
        assert got == r, (key, got, r)
        assert po.crdt_value(typ, got[1]) == want


@pytest.mark.parametrize("c", TXN, ids=[c["name"] for c in TXN])
def test_system_txn(oracle_lib, c):
    system_txn_check(c, oracle_fn(oracle_lib))
