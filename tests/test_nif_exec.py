"""The NIF's own C (nif/antidote_gpu_nif.c) executed on the GPU through the
minimal erl_nif runtime (tests/nif_rt, test infrastructure): the functions an
Erlang node calls -- part_open / part_update / part_read / part_store /
part_gc_due / part_key_meta / part_stats, materialize/6, gst_min/5 -- with
Erlang terms in and out (keys, DC ids, TxIds, effects, orddict states),
checked against:

  * the Python twin of the partition (test_typed_partition.TypedPartition:
    the same C-ABI calls made from Python), read for read over a workload of
    keys of all three CRDT types in one partition with mis-typed writes and
    reads -- every value served and every corrupted_ops_cache raised
    (src/clocksi_materializer.erl:190-191), and the ETS meta (Length,
    ListLen, op id) of every key;
  * agn_materialize_host for materialize/6 (the per-call path) and the C
    oracle for gst_min/5;
  * the reference's error convention for an effect the CRDT rejects:
    {error, {unexpected_operation, Op, Type}} with the very effect term
    (src/materializer.erl:51-58);
  * the partition resource's destructor (device logs freed when the last
    reference goes).

The Erlang half of the drop-in (nif/antidote_gpu_nif.erl: update/3's GC read
before the insert, read/5's log fallback through part_store/8) is mirrored by
NifPart below, as test_ss_states.NifPartition mirrors it for the twin.
"""
import os
import sys

import numpy as np
import pytest

from antidote_amd import _abi
from antidote_amd import clocksi_materializer as cm
from antidote_amd.encode import alloc_result
from oracle import py_oracle as po
from synth import compare, random_case
from test_ss_states import PTYPE, log_response, vc
from test_typed_partition import TYPES, MixedWorkload, TypedPartition

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "nif_rt"))
import terms  # noqa: E402
from terms import Atom, NifRaise  # noqa: E402

pytestmark = pytest.mark.gpu

TYPE_ATOM = {_abi.COUNTER_PN: Atom("antidote_crdt_counter_pn"),
             _abi.SET_AW: Atom("antidote_crdt_set_aw"),
             _abi.REGISTER_MV: Atom("antidote_crdt_register_mv")}
OK, ERROR, IGNORE = Atom("ok"), Atom("error"), Atom("ignore")


def dc(d):
    """A dcid() term ({atom(), tuple()}, include/antidote.hrl:187)."""
    return (Atom(f"antidote_{d}@127.0.0.1"), (1700, 0, d))


def pairs(row):
    return [(dc(d), int(t)) for d, t in enumerate(row)]


def dict_pairs(clock):
    return [(dc(d), int(t)) for d, t in sorted(clock.items())]


@pytest.fixture(scope="module")
def nif():
    terms.build()
    rt = terms.NifRuntime()
    r = rt.call("open", 0, keep=True)
    assert r[0] == OK, r
    yield rt, r[1]
    rt.release_all()


class NifPart:
    """A cached partition through the NIF, driven as nif/antidote_gpu_nif.erl
    drives it: update/3 (part_gc_due -> GC part_read -> on no_snapshot the
    log read + part_store with Gc -> part_update) and read/5 (part_read ->
    on no_snapshot the log read)."""

    def __init__(self, rt, ctx, d, K, first):
        self.rt, self.d = rt, d
        r = rt.call("part_open", ctx, TYPE_ATOM[first], d, K, True, keep=True)
        assert r[0] == OK, r
        self.part, self.ref = r[1], rt.kept[-1]
        self.disk = []

    def close(self):
        """Drop the test's reference: the partition's destructor runs (its
        device logs, batchers and scratch are freed)."""
        self.rt.kept.remove(self.ref)
        self.rt.lib.rt_release(self.ref)

    def call(self, name, *args):
        try:
            return self.rt.call(name, self.part, *args)
        except NifRaise as e:
            if e.reason == Atom("corrupted_ops_cache"):
                raise po.CorruptedOpsCache() from None
            raise

    def from_log(self, key, t, R_dict, gc):
        counter = t == _abi.COUNTER_PN
        resp = log_response(self.disk, key, R_dict, 0 if counter else None)
        if resp.number_of_ops == 0:
            return ("ok", 0 if counter else [])
        r = cm.materialize(PTYPE[t], po.IGNORE, R_dict, resp)
        if r[0] != "ok":
            return r
        _, value, hole, ct, _newss, count = r
        if gc and ct != po.IGNORE:
            term = value if counter else (
                [(e, list(ts)) for e, ts in value] if t == _abi.SET_AW else [tuple(p) for p in value])
            assert self.call("part_store", key, TYPE_ATOM[t], dict_pairs(ct), int(hole), int(count),
                             term, True) == OK
        return ("ok", value)

    def update(self, key, t, pay, oc, eff, entry, txid):
        self.disk.append(pay)
        ta = TYPE_ATOM[t]
        if self.call("part_gc_due", key, ta) == Atom("true"):
            g = self.call("part_read", key, ta, dict_pairs(pay.snapshot_time), IGNORE, True)
            if g == (ERROR, Atom("no_snapshot")):
                self.from_log(key, t, pay.snapshot_time, True)
            else:
                assert g[0] == OK, g
        effect = eff if t != _abi.REGISTER_MV else tuple(eff)
        r = self.call("part_update", key, ta, pairs(oc), txid, effect)
        assert r[0] == OK, r
        return r

    def read(self, key, t, R):
        g = self.call("part_read", key, TYPE_ATOM[t], pairs(R), IGNORE, False)
        if g == (ERROR, Atom("no_snapshot")):
            return self.from_log(key, t, vc(R), False)
        assert g[0] == OK and len(g) == 6, g
        return ("ok", g[1])

    def key_meta(self, key, t):
        return tuple(self.call("part_key_meta", key, TYPE_ATOM[t]))


def norm(t, v):
    """A served value in one form for both sides: counter int, set_aw
    [(elem, [tokens])], register_mv sorted [(value, token)]."""
    if v in ("corrupted",):
        return v
    tag, val = v
    if t == _abi.COUNTER_PN:
        return (tag, int(val))
    if t == _abi.SET_AW:
        return (tag, [(int(e), [int(x) for x in ts]) for e, ts in val])
    return (tag, sorted((int(a), int(b)) for a, b in val))


@pytest.mark.parametrize("seed", [1, 2])
def test_nif_partition_vs_twin(eng, nif, seed):
    """update/2 + read/6 over one partition holding keys of every type (keys
    0..2 get the odd op of another type; 8 % of the reads of a cached key use
    another type): the NIF and its Python twin serve every read identically
    -- the value, or corrupted_ops_cache -- and keep the same (Length,
    ListLen, op id) for every key and type."""
    rt, ctx = nif
    d, K, steps = 4, 12, 1500
    nominal = {k: TYPES[k % 3] for k in range(K)}
    w = MixedWorkload(300 + seed, K, d)
    twin = TypedPartition(eng, d, K, _abi.COUNTER_PN)
    part = NifPart(rt, ctx, d, K, _abi.COUNTER_PN)
    n_res = rt.live_resources()
    closed = False
    served = raised = 0
    try:
        for s in range(steps):
            key = int(w.rng.integers(0, K))
            if w.rng.random() < 0.65:
                t = nominal[key]
                if key < 3 and w.rng.random() < 0.04:
                    t = TYPES[(TYPES.index(t) + 1 + int(w.rng.integers(0, 2))) % 3]
                c, ss, ct, oc, eff, entry = w.op(key, t)
                pay = po.Payload(key, PTYPE[t], eff, vc(ss), (c, ct), s + 1)
                outs = []
                for side in (twin, part):
                    try:
                        side.update(key, t, pay, oc, eff, entry, s + 1)
                        outs.append("ok")
                    except po.CorruptedOpsCache:
                        outs.append("corrupted")
                assert outs[0] == outs[1], (s, key, t, outs)
            else:
                t = nominal[key]
                if w.rng.random() < 0.08:
                    t = TYPES[(TYPES.index(t) + 1) % 3]
                R = w.read_clock(lag=400 if w.rng.random() < 0.85 else 20000)
                got = []
                for side in (twin, part):
                    try:
                        got.append(norm(t, side.read(key, t, R)))
                    except po.CorruptedOpsCache:
                        got.append("corrupted")
                assert got[0] == got[1], (s, key, t, got)
                served += got[0] != "corrupted"
                raised += got[0] == "corrupted"
        for t, p in twin.sub.items():
            ln, ll, ct = p.ol.key_meta()
            for k in range(K):
                assert part.key_meta(k, t) == (int(ln[k]), int(ll[k]), int(ct[k])), (t, k)
        e, sl, tk = part.call("part_stats")
        assert e == sum(p.ol.stats()["entries"] for p in twin.sub.values())
        # the partition's last reference: its destructor runs
        part.close()
        closed = True
        assert rt.live_resources() == n_res - 1
    finally:
        twin.close()
        if not closed:
            part.close()
    assert served > 300 and raised > 10, (served, raised)


def ctx_of(nif):
    return nif[1]


def test_nif_unexpected_operation_and_type_errors(eng, nif):
    """A counter effect the CRDT rejects (an atom) is stored as an invalid op:
    the read returns {error, {unexpected_operation, Effect, Type}} with the
    very term; reading the key as another type raises corrupted_ops_cache;
    a never-written key of a type with no log reads as Type:new()."""
    rt = nif[0]
    part = NifPart(rt, ctx_of(nif), 3, 8, _abi.COUNTER_PN)
    try:
        _unexpected_operation_body(part)
    finally:
        part.close()


def _unexpected_operation_body(part):
    ta = TYPE_ATOM[_abi.COUNTER_PN]
    for i, e in enumerate([5, 7, Atom("bogus"), 11]):
        r = part.call("part_update", 0, ta, pairs([100 + i, 50, 50]), i + 1, e)
        assert r[0] == OK and r[1] == i + 1, r
    for i in range(3):
        part.call("part_update", 1, ta, pairs([200 + i, 60, 60]), 10 + i, 2)
    R = pairs([10 ** 6] * 3)
    assert part.call("part_read", 0, ta, R, IGNORE, False) == \
        (ERROR, (Atom("unexpected_operation"), Atom("bogus"), ta))
    # a snapshot that excludes the invalid op is served
    g = part.call("part_read", 0, ta, pairs([101, 50, 50]), IGNORE, False)
    assert g == (ERROR, Atom("no_snapshot")) or g[:2] == (OK, 12), g
    g = part.call("part_read", 1, ta, R, IGNORE, False)
    assert g[0] == OK and g[1] == 6 and g[5] == 3, g
    with pytest.raises(po.CorruptedOpsCache):
        part.call("part_read", 1, TYPE_ATOM[_abi.SET_AW], R, IGNORE, False)
    g = part.call("part_read", 5, TYPE_ATOM[_abi.REGISTER_MV], R, IGNORE, False)
    assert g == (OK, [], 0, IGNORE, Atom("false"), 0), g
    assert part.call("part_gc_due", 0, ta) in (Atom("true"), Atom("false"))
    # malformed terms are badarg, never a crash
    with pytest.raises(terms.NifBadarg):
        part.call("part_update", 0, ta, [(dc(0),)], 1, 1)
    with pytest.raises(terms.NifBadarg):
        part.call("part_read", 0, Atom("antidote_crdt_bogus"), R, IGNORE, False)


@pytest.mark.parametrize("crdt", [_abi.COUNTER_PN, _abi.SET_AW, _abi.REGISTER_MV])
def test_nif_materialize_per_call(eng, nif, crdt):
    """materialize/6 (the per-call path the Erlang module's materialize/4
    encodes for) on a random batch: every result binary equals
    agn_materialize_host's for the same arrays."""
    rt = nif[0]
    D = 5
    log, req, cap = random_case(71 + crdt, crdt, 60, D, 40, sparse=True, warm=0.3, txid=0.2,
                                base=0.3 if crdt != _abi.COUNTER_PN else 0.0)
    want = eng.materialize_host(log, req, sparse=True, cap_off=cap)

    def b(a):
        return b"" if a is None else np.ascontiguousarray(a).tobytes()
    L = (b(log.key_off), b(getattr(log, "key_type", None)), b(log.oc), b(log.oc_mask),
         b(log.op_id), b(log.txid), b(log.eff), b(log.tag), b(log.add_tok), b(log.rem_off),
         b(log.rem_tok))
    Q = (b(req.keys), b(req.R), b(req.R_mask), b(req.sct), b(req.sct_mask), b(req.sct_ignore),
         b(req.txid), b(req.base_value), b(req.base_off), b(req.base_tag), b(req.base_tok))
    r = rt.call("materialize", ctx_of(nif), crdt, D, L, Q, b(cap))
    assert r[0] == OK, r
    value, hole, lastct, lastct_mask, count, flags, err_pos, out_n, out_tag, out_tok = r[1]
    n = req.n_req
    got = alloc_result(n, D, sparse=True, cap_off=cap)
    got.value[:] = np.frombuffer(value, np.int64)[:n]
    got.hole[:] = np.frombuffer(hole, np.int64)[:n]
    got.lastct[:] = np.frombuffer(lastct, np.uint64)[:n * D].reshape(n, D)
    got.lastct_mask[:] = np.frombuffer(lastct_mask, np.uint64)[:got.lastct_mask.size].reshape(
        got.lastct_mask.shape)
    got.count[:] = np.frombuffer(count, np.uint32)[:n]
    got.flags[:] = np.frombuffer(flags, np.uint32)[:n]
    got.err_pos[:] = np.frombuffer(err_pos, np.uint32)[:n]
    if crdt != _abi.COUNTER_PN:
        got.out_n[:] = np.frombuffer(out_n, np.uint32)[:n]
        m = got.out_tag.size
        got.out_tag[:] = np.frombuffer(out_tag, np.uint32)[:m]
        got.out_tok[:] = np.frombuffer(out_tok, np.uint64)[:m]
    bad = compare(crdt, D, got, want, True, n)
    assert not bad, bad[:5]


def test_nif_gst_min(eng, nif, oracle_lib):
    """gst_min/5 (stable_time_functions:get_min_time/1 on the device) against
    the oracle, with an undefined partition and without."""
    rt = nif[0]
    rng = np.random.default_rng(9)
    D, P = 7, 33
    clocks = rng.integers(1, 10 ** 9, (P, D)).astype(np.uint64)
    clocks[3, 2] = np.uint64(2 ** 64 - 1)       # a DC absent from one entry
    for undefined in (False, True):
        defined = np.ones(P, np.uint8)
        if undefined:
            defined[5] = 0
        r = rt.call("gst_min", ctx_of(nif), D, P, clocks.tobytes(), defined.tobytes())
        assert r[0] == OK, r
        got = np.frombuffer(r[1], np.uint64)
        want = np.zeros(D + 1, np.uint64)
        assert oracle_lib.oracle_gst_min(D, P, 1, clocks.ctypes.data, defined.ctypes.data,
                                         want.ctypes.data, 1) == 0
        assert np.array_equal(got, want), (undefined, got, want)
