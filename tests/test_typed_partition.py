"""One partition holding keys of every CRDT type, as the reference's
ops_cache-<P> does (src/materializer_vnode.erl:284-286, 321-338, 621-647).

nif/antidote_gpu_nif.c keeps one engine-owned op log (+ cached read batcher)
per CRDT type inside a partition resource, created with the type's first op.
A read of a key that holds ops of another type raises corrupted_ops_cache,
as materialize_intern's type check does (src/clocksi_materializer.erl:
190-191); a read of a type the partition has no log for yet is
materialize/4 over no ops (Type:new()).  TypedPartition below makes exactly
the C-ABI calls the NIF makes (agn_oplog_* / agn_batcher_* through
antidote_amd.engine, the log fallback of test_ss_states.NifPartition), and
the sequence is replayed against the reference's ETS transcription
(oracle/py_oracle.MaterializerVnode, one ops cache for every type).
"""
import numpy as np
import pytest

from antidote_amd import _abi
from antidote_amd.engine import Batcher, OpLog
from oracle import py_oracle as po
from test_ss_states import PTYPE, NifPartition, state_of, vc

pytestmark = pytest.mark.gpu

TYPES = (_abi.COUNTER_PN, _abi.SET_AW, _abi.REGISTER_MV)


class TypedPartition:
    """The NIF's partition resource over the C ABI (part_update/6,
    part_read/6 with the log fallback of antidote_gpu_nif.erl read/5)."""

    def __init__(self, eng, d, K, first):
        self.eng, self.d, self.K = eng, d, K
        self.full = np.uint64((1 << d) - 1)
        self.disk = []          # the logging_vnode's committed payloads, every type
        self.sub = {}
        # the reference's one ETS tuple per key: one op counter across the
        # per-type logs and the home type (its first op's), whose log holds
        # the tuple's ListLen (the NIF's kcnt / khome)
        self.kcnt, self.khome = {}, {}
        self.make(first)

    def make(self, t):          # sub_make: the type's log with its first op
        if t not in self.sub:
            ol = OpLog(self.eng, t, self.d, self.K, sparse=True)
            bt = Batcher(ol, max_batch=8, cached=True)
            part = NifPartition(ol, bt, t, self.d, True)
            part.disk = self.disk
            self.sub[t] = part
        return self.sub[t]

    def close(self):
        for p in self.sub.values():
            p.bt.close()
            p.ol.close()

    def other_type_ops(self, key, t):
        return any(int(p.ol.key_meta()[0][key]) != 0 for u, p in self.sub.items() if u != t)

    def gc_due(self, key):
        """op_insert_gc's trigger (:635) on the key's one tuple: Length = its
        ops of every type, ListLen = the home type's log's, NewId = the shared
        counter + 1 (part_gc_due/3)."""
        if key not in self.khome:
            return False
        total = sum(int(p.ol.key_meta([key])[0][0]) for p in self.sub.values())
        lcap = int(self.sub[self.khome[key]].ol.key_meta([key])[1][0])
        return total >= max(lcap, _abi.OPS_THRESHOLD) or \
            (self.kcnt[key] + 1) % _abi.OPS_THRESHOLD == 0

    def update(self, key, t, pay, oc, eff, entry, txid):
        self.disk.append(pay)                   # logged before the materializer
        p = self.make(t)
        if self.gc_due(key):                    # op_insert_gc's GC read (:640)
            if self.other_type_ops(key, t):
                # part_read raises; nothing inserted, but the op's id was
                # taken (:630 precedes the read)
                self.kcnt[key] += 1
                raise po.CorruptedOpsCache()
            g = p.bt.read(key, R=pay_row(pay, self.d), R_mask=np.array([self.full]), gc=True,
                          out_cap=4096)
            if g["status"] == _abi.SS_LOG:
                p.from_log(key, pay.snapshot_time, True)
        p.ol.set_counter(key, self.kcnt.get(key, 0))
        keys = np.array([key], np.uint64)
        oc1 = oc.reshape(1, self.d).astype(np.uint64)
        mask = np.array([[self.full]], np.uint64)
        if t == _abi.COUNTER_PN:
            ids, _ = p.ol.append(keys, oc1, oc_mask=mask, eff=np.array([eff], np.int64),
                                 txid=np.array([txid], np.uint64))
        else:
            tag, add, rems = entry
            ids, _ = p.ol.append(keys, oc1, oc_mask=mask, tag=np.array([tag], np.uint32),
                                 add_tok=np.array([add], np.uint64),
                                 rem_off=np.array([0, len(rems)], np.uint32),
                                 rem_tok=np.array(rems if rems else [0], np.uint64),
                                 txid=np.array([txid], np.uint64))
        self.kcnt[key] = int(ids[0])
        self.khome.setdefault(key, t)

    def read(self, key, t, R):
        if self.other_type_ops(key, t):
            raise po.CorruptedOpsCache()
        if t not in self.sub:                   # no log of the type: Type:new()
            return ("ok", 0 if t == _abi.COUNTER_PN else [])
        p = self.sub[t]
        g = p.bt.read(key, R=R.astype(np.uint64), R_mask=np.array([self.full]), out_cap=4096)
        if g["status"] == _abi.SS_LOG:
            p.log_reads += 1
            return p.from_log(key, vc(R), False)
        if t == _abi.COUNTER_PN:
            return ("ok", g["value"])
        return ("ok", state_of(t, g["out_tag"], g["out_tok"]))


def pay_row(pay, d):
    row = np.zeros(d, np.uint64)
    for dc, tm in pay.snapshot_time.items():
        row[dc] = tm
    return row


class MixedWorkload:
    """One causal clock for every key; each key has a type (its bucket's),
    and now and then an op of another type lands on it (the mis-typed write
    the reference's type check catches)."""

    def __init__(self, seed, K, d):
        self.rng = np.random.default_rng(seed)
        self.d = d
        self.clk = np.full(d, 1000, np.int64)
        self.live = [dict() for _ in range(K)]
        self.tok = 1

    def op(self, key, t):
        d = self.d
        c = int(self.rng.integers(0, d))
        ss = np.maximum(self.clk - self.rng.integers(0, 40, d), 0)
        self.clk[c] += int(self.rng.integers(1, 30))
        oc = ss.copy()
        oc[c] = self.clk[c]
        live = self.live[key]
        if t == _abi.COUNTER_PN:
            e = int(self.rng.integers(-50, 51))
            return c, ss, int(self.clk[c]), oc, e, None
        if t == _abi.SET_AW:
            el = int(self.rng.integers(0, 6))
            obs = list(live.get(el, []))
            if self.rng.random() < 0.75:
                tk = self.tok
                self.tok += 1
                live[el] = [tk]
                return c, ss, int(self.clk[c]), oc, [(el, [tk], obs)], (el, tk, obs)
            live[el] = []
            return c, ss, int(self.clk[c]), oc, [(el, [], obs)], (el, 0, obs)
        obs = [x for ts in live.values() for x in ts]
        v, tk = int(self.rng.integers(0, 5)), self.tok
        self.tok += 1
        live.clear()
        live[0] = [tk]
        return c, ss, int(self.clk[c]), oc, (v, tk, obs), (v, tk, obs)

    def read_clock(self, lag=400):
        return np.maximum(self.clk - self.rng.integers(0, lag, self.d), 0)


def test_counter_key_read_as_set(eng):
    """The minimal case: a key written as counter_pn and read as set_aw raises
    corrupted_ops_cache on both sides; read as counter_pn it is served; a key
    never written reads as Type:new().  (A key's first read stores the empty
    snapshot of the read's type, get_from_snapshot_cache :388-397, so the
    counter key is read as a counter first; see test_typed_partition_vs_reference
    for the reference's cache poisoning by a mis-typed first read.)"""
    d, K = 3, 5
    vn = po.MaterializerVnode(disk_log=True)
    part = TypedPartition(eng, d, K, _abi.COUNTER_PN)
    w = MixedWorkload(7, K, d)
    try:
        total = 0
        for s in range(12):
            c, ss, ct, oc, eff, _ = w.op(0, _abi.COUNTER_PN)
            pay = po.Payload(0, po.COUNTER_PN, eff, vc(ss), (c, ct), s + 1)
            vn.update(0, pay)
            part.update(0, _abi.COUNTER_PN, pay, oc, eff, None, s + 1)
            total += eff
        R = w.clk.copy()
        assert vn.read(0, po.COUNTER_PN, vc(R), po.IGNORE) == ("ok", total)
        assert part.read(0, _abi.COUNTER_PN, R) == ("ok", total)
        for t in (_abi.SET_AW, _abi.REGISTER_MV):
            with pytest.raises(po.CorruptedOpsCache):
                vn.read(0, PTYPE[t], vc(R), po.IGNORE)
            with pytest.raises(po.CorruptedOpsCache):
                part.read(0, t, R)
        assert vn.read(0, po.COUNTER_PN, vc(R), po.IGNORE) == ("ok", total)
        assert part.read(0, _abi.COUNTER_PN, R) == ("ok", total)
        for k, t in zip((1, 2, 3), TYPES):   # never written, one type each
            want = vn.read(k, PTYPE[t], vc(R), po.IGNORE)
            assert part.read(k, t, R) == want == ("ok", 0 if t == _abi.COUNTER_PN else [])
    finally:
        part.close()


@pytest.mark.parametrize("seed", [1, 2])
def test_typed_partition_vs_reference(eng, seed):
    """update/2 and read/6 over keys of all three types in one partition:
    keys 0..2 now and then get an op of another type (the mis-typed write the
    reference's type check catches), and 8 % of the reads of a key that has a
    cached snapshot use another type than the key's.  Every read is served
    or raised exactly as the transcription's (value, or corrupted_ops_cache),
    and the ETS list sizes follow it slot for slot on single-typed keys.

    The partition keeps the reference's one tuple per key across its
    per-type logs (one op counter, the GC trigger on the key's ops of every
    type, the op id consumed by a GC read that raises): every update fires
    and raises exactly as the transcription's (`diverged` stays empty).
    Not replicated (intentional): (1) the reference's first
    read of a key stores the empty snapshot of the READ's type
    (get_from_snapshot_cache :388-397), so a mis-typed first read leaves a
    base of the wrong type under the key's later reads; here a mis-typed read
    raises or returns Type:new() without touching another type's cache.  Keys
    whose reference cache was seeded that way leave the comparison
    (`quirk`).  (2) A read that no cached snapshot serves goes to the log in
    the reference, and when the log holds no op of the key at or below R,
    materialize_snapshot returns Type:new() without visiting an op
    (:469-473): no type check.  The partition raises corrupted_ops_cache for
    such a read of a key holding ops of another type; such reads are counted
    (`mistyped_log_reads`) and checked to be exactly that case.  Every count
    is pinned (EXPECT)."""
    d, K, steps = 4, 12, 2500
    nominal = {k: TYPES[k % 3] for k in range(K)}
    w = MixedWorkload(100 + seed, K, d)
    vn = po.MaterializerVnode(disk_log=True)
    part = TypedPartition(eng, d, K, _abi.COUNTER_PN)
    mixed, quirk, diverged = set(), set(), set()
    served = raised = log_typed = 0
    try:
        for s in range(steps):
            key = int(w.rng.integers(0, K))
            if w.rng.random() < 0.65:
                t = nominal[key]
                if key < 3 and w.rng.random() < 0.04:
                    t = TYPES[(TYPES.index(t) + 1 + int(w.rng.integers(0, 2))) % 3]
                    mixed.add(key)
                c, ss, ct, oc, eff, entry = w.op(key, t)
                pay = po.Payload(key, PTYPE[t], eff, vc(ss), (c, ct), s + 1)
                ref_err = got_err = None
                cached = key in vn.snapshot_cache
                try:
                    vn.update(key, pay)
                except po.CorruptedOpsCache as e:   # the reference vnode's GC read crashes
                    ref_err = e
                except po.BadMatch:
                    quirk.add(key)
                if not cached and key in vn.snapshot_cache and t != nominal[key]:
                    quirk.add(key)                  # a base of the op's type stored
                try:
                    part.update(key, t, pay, oc, eff, entry, s + 1)
                except po.CorruptedOpsCache as e:
                    got_err = e
                if (ref_err is None) != (got_err is None):
                    # the GC trigger follows the reference's one tuple per key
                    # (shared op counter / Length / ListLen): no divergence
                    # is expected; one would show in EXPECT
                    assert key in mixed, (s, key)
                    diverged.add(key)
                tup = vn.ops_cache.get(key)
                if tup and any(tup[po.FIRST_OP - 1 + i] == 0 for i in range(tup[1][0])):
                    quirk.add(key)
            else:
                t = nominal[key]
                if key in vn.snapshot_cache and w.rng.random() < 0.08:
                    t = TYPES[(TYPES.index(t) + 1) % 3]
                R = w.read_clock(lag=400 if w.rng.random() < 0.85 else 20000)
                # served from the log with no op at or below R: the reference
                # never visits an op, so never checks a type (see the docstring)
                log_empty = (key in vn.snapshot_cache and
                             vn.snapshot_cache[key].get_smaller(vc(R))[0] is None and
                             not any(p.key == key and po.vc_le(p.snapshot_time, vc(R))
                                     for p in vn.disk_log))
                try:
                    want = vn.read(key, PTYPE[t], vc(R), po.IGNORE)
                except po.CorruptedOpsCache:
                    want = "corrupted"
                except po.BadMatch:
                    quirk.add(key)
                    continue
                try:
                    got = part.read(key, t, R)
                except po.CorruptedOpsCache:
                    got = "corrupted"
                if key in quirk or key in diverged:
                    continue
                # (a key holding ops of two types: a read of either type)
                if log_empty and (t != nominal[key] or key in mixed) and got == "corrupted":
                    assert want == ("ok", 0 if t == _abi.COUNTER_PN else []), (s, key, want)
                    log_typed += 1
                    continue
                assert got == want, (s, key, t, want, got)
                served += got != "corrupted"
                raised += got == "corrupted"
        for t, p in part.sub.items():
            ln, ll, _ = p.ol.key_meta()
            for k in range(K):
                if k in mixed or k in quirk or nominal[k] != t or k not in vn.ops_cache:
                    continue
                assert (int(ln[k]), int(ll[k])) == tuple(vn.ops_cache[k][1]), (t, k)
    finally:
        part.close()
    got = dict(served=served, raised=raised, mixed=len(mixed), diverged=len(diverged),
               quirk=len(quirk), mistyped_log_reads=log_typed)
    print(" ".join(f"{k}={v}" for k, v in got.items()))
    # the workload is deterministic: every count -- the excluded keys included
    # (`diverged` only ever holds keys that got an op of another type, asserted
    # above) -- is pinned, so a regression that moved a key in or out of the
    # comparison shows (profiles/r06: the GPU run that recorded them)
    assert got == EXPECT[seed], (got, EXPECT[seed])


EXPECT = {1: dict(served=662, raised=203, mixed=3, diverged=0, quirk=0, mistyped_log_reads=6),
          2: dict(served=631, raised=234, mixed=3, diverged=0, quirk=0, mistyped_log_reads=5)}
