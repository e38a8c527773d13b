"""The drop-in's call sequence (what the NIF does for materializer_vnode,
SURVEY.md §8(b) Ownership / Threading) replayed through the C ABI:

  update/2  -> agn_oplog_append (op ids, op_insert_gc's GC trigger) and, when
               due, the GC read (agn_batcher_read with AGN_READ_GC);
  read/6    -> agn_batcher_read on a cached batcher: the fused one-kernel
               batch (read6.hip: lookup -> materialize -> store) or, with
               AGN_READ6=0, agn_ss_lookup -> agn_materialize -> agn_ss_store;
               then the in-place GC of the batch's selected keys.

Sequentially, every read must equal the reference's transcription
(oracle/py_oracle.MaterializerVnode: ETS ops tuple, snapshot cache, GC,
resize), including whether the snapshot cache can serve it at all.  With a
writer thread and 8 reader threads, every served read must equal the value
of the key's ops at R (whatever the cache held and whatever GC ran)."""
import threading

import numpy as np
import pytest

from antidote_amd import _abi, _lib
from antidote_amd.engine import Batcher, OpLog
from oracle import py_oracle as po

pytestmark = pytest.mark.gpu

D = 3
BIG = 10 ** 15


def vc(row, mask=None):
    return {d: int(row[d]) for d in range(len(row)) if mask is None or (int(mask) >> d) & 1}


class Workload:
    """Per-DC clocks that only grow; an op commits at DC c after the others'
    current times (its snapshot), so op clocks are causal and reads at any
    R <= the current clocks see exactly the ops already appended."""

    def __init__(self, seed, K, d=D):
        self.rng = np.random.default_rng(seed)
        self.K, self.D = K, d
        self.clk = np.full(d, 1000, np.int64)
        self.ops = [[] for _ in range(K)]   # per key: (oc row, eff)

    def op(self, key):
        D = self.D
        c = int(self.rng.integers(0, D))
        ss = self.clk - self.rng.integers(0, 40, D)
        ss = np.maximum(ss, 0)
        self.clk[c] += int(self.rng.integers(1, 30))
        ct = int(self.clk[c])
        oc = ss.copy()
        oc[c] = ct
        eff = int(self.rng.integers(-50, 51))
        return c, ss, ct, oc, eff

    def read_clock(self, lag=400):
        return np.maximum(self.clk - self.rng.integers(0, lag, self.D), 0)


def has_placeholder(vn, key):
    """The reference's all-pruned quirk: prune_ops keeps element(?FIRST_OP+Len),
    an empty slot (0), as the only op (src/materializer_vnode.erl:580-583); the
    engine keeps zero entries instead (AGN_GC_ALL_PRUNED)."""
    tup = vn.ops_cache.get(key)
    if tup is None:
        return False
    length = tup[1][0]
    return any(tup[po.FIRST_OP - 1 + i] == 0 for i in range(length))


def engine_update(ol, bt, key, ss, oc, eff, txid, mask=None):
    """op_insert_gc/3 (:621-647) in the reference's order: the GC read at the
    op's snapshot time (:640) when due, then the insert.  mask: the op's DC
    set (a presence-masked log)."""
    m = None if mask is None else np.array([mask], np.uint64)
    if ol.gc_due(key)[0]:
        bt.read(key, R=ss.astype(np.uint64), R_mask=m, gc=True)
    ids, _ = ol.append(np.array([key], np.uint64), oc.reshape(1, len(oc)).astype(np.uint64),
                       oc_mask=None if m is None else m.reshape(1, 1),
                       eff=np.array([eff], np.int64), txid=np.array([txid], np.uint64))
    return int(ids[0])


# D <= 8: read6.hip k_read6 (register-resident clocks); D = 16 / 64: k_read6w
# (the general per-key filter between the cache lookup and store)
@pytest.mark.parametrize("d", [3, 16, 64])
@pytest.mark.parametrize("read6", ["1", "0"])
def test_vnode_replay_sequential_vs_reference(eng, monkeypatch, read6, d):
    monkeypatch.setenv("AGN_READ6", read6)
    K, steps = 24, 4000
    w = Workload(11 + d, K, d)
    vn = po.MaterializerVnode()
    quirk = set()   # keys where the reference hit the all-pruned placeholder (:580-583)
    served = log_reads = 0
    with OpLog(eng, _abi.COUNTER_PN, d, K) as ol, \
            Batcher(ol, max_batch=8, cached=True) as bt:
        for s in range(steps):
            key = int(w.rng.integers(0, K))
            if w.rng.random() < 0.7:
                c, ss, ct, oc, eff = w.op(key)
                pay = po.Payload(key, po.COUNTER_PN, eff, vc(ss), (c, ct), s + 1)
                try:
                    vn.update(key, pay)
                except po.BadMatch:
                    quirk.add(key)
                engine_update(ol, bt, key, ss, oc, eff, s + 1)
                w.ops[key].append((oc, eff))
                if has_placeholder(vn, key):
                    quirk.add(key)
            else:
                # mostly recent reads; some far in the past (older than every
                # cached snapshot once GC has run: the log fallback)
                R = w.read_clock(lag=400 if w.rng.random() < 0.85 else 20000)
                g = bt.read(key, R=R.astype(np.uint64))
                if key in quirk:
                    continue
                try:
                    want = vn.read(key, po.COUNTER_PN, vc(R), po.IGNORE)
                except NotImplementedError:      # get_from_snapshot_log
                    assert g["status"] == _abi.SS_LOG, (s, key)
                    log_reads += 1
                    continue
                except po.BadMatch:
                    quirk.add(key)
                    continue
                assert g["status"] in (_abi.SS_HIT, _abi.SS_NEW), (s, key, g["status"])
                assert want == ("ok", g["value"]), (s, key, want, g["value"])
                served += 1
                if has_placeholder(vn, key):
                    quirk.add(key)
        ln, ll, ct = ol.key_meta()
    # (at D = 64 a read's clock is rarely below every kept snapshot within
    # the run: the log fallback is exercised at the narrower widths)
    assert served > 1000 and (log_reads > 0 or d > 16)
    assert len(quirk) < K // 2
    for k in range(K):
        if k in quirk or k not in vn.ops_cache:
            continue
        length, list_len = vn.ops_cache[k][1]
        assert (int(ln[k]), int(ll[k]), int(ct[k])) == (length, list_len, vn.ops_cache[k][2]), k


@pytest.mark.parametrize("d", [3, 16, 64])
@pytest.mark.parametrize("read6", ["1", "0"])
def test_vnode_replay_threads_values(eng, monkeypatch, read6, d):
    """1 writer (the vnode: update/2 + GC reads) and 8 read servers."""
    monkeypatch.setenv("AGN_READ6", read6)
    K = 16
    w = Workload(5 + d, K, d)
    lock = threading.Lock()
    errs, stats = [], {"served": 0, "log": 0}
    with OpLog(eng, _abi.COUNTER_PN, d, K, init_slots=8) as ol, \
            Batcher(ol, max_batch=16, max_wait_us=100, cached=True) as bt:
        stop = threading.Event()

        readers_done = threading.Event()

        def writer():
            try:
                for s in range(20_000):
                    if readers_done.is_set() and s >= 3000:
                        break
                    key = s % K if s < K else int(w.rng.integers(0, K))
                    # the clocks a reader may pick advance only with the append
                    with lock:
                        c, ss, ct, oc, eff = w.op(key)
                        engine_update(ol, bt, key, ss, oc, eff, s + 1)
                        w.ops[key].append((oc, eff))
            except Exception as e:  # noqa: BLE001
                errs.append(e)
            finally:
                stop.set()

        def reader(t):
            rng = np.random.default_rng(100 + t)
            try:
                for _ in range(60):
                    if errs:
                        break
                    key = int(rng.integers(0, K))
                    with lock:
                        # ops at or below the published clocks are all appended
                        R = np.maximum(w.clk - rng.integers(0, 300, d), 0)
                    g = bt.read(key, R=R.astype(np.uint64))
                    with lock:
                        ops = list(w.ops[key])
                    if g["status"] == _abi.SS_LOG:
                        stats["log"] += 1
                        continue
                    want = sum(e for oc, e in ops if (oc <= R).all())
                    assert g["value"] == want, (key, g["value"], want)
                    stats["served"] += 1
            except Exception as e:  # noqa: BLE001
                errs.append(e)
        rs = [threading.Thread(target=reader, args=(t,)) for t in range(8)]
        wt = threading.Thread(target=writer)
        wt.start()
        for x in rs:
            x.start()
        for x in rs:
            x.join()
        readers_done.set()
        wt.join()
        assert not errs, errs[0]
        # after the storm: every key read at the current clocks, served
        for key in range(K):
            g = bt.read(key, R=w.clk.astype(np.uint64))
            assert g["status"] in (_abi.SS_HIT, _abi.SS_NEW)
            assert g["value"] == sum(e for _, e in w.ops[key])
        st = ol.stats()
    assert stats["served"] > 100, stats
    assert st["entries"] < sum(len(x) for x in w.ops)   # the GC ran


def rand_mask(rng, d):
    return int(sum(int(b) << i for i, b in enumerate(rng.integers(0, 2, d))))


class CounterNifPartition:
    """A cached counter partition driven the way nif/antidote_gpu_nif.erl
    drives it (test_ss_states.NifPartition for counters): update/2 runs
    op_insert_gc's GC read first when due, and a read (GC or not) that no
    cached snapshot serves goes to the partition's log -- materialize/4 of
    get_from_snapshot_log's response, and for a GC read the result stored on
    the device cache (agn_batcher_store)."""

    def __init__(self, ol, bt, d):
        from test_ss_states import NifPartition
        self.p = NifPartition(ol, bt, _abi.COUNTER_PN, d, True)

    def update(self, key, pay, ss, oc, eff, txid, mask):
        p = self.p
        p.disk.append(pay)                       # logged before the materializer
        m = np.array([mask], np.uint64)
        if p.ol.gc_due(key)[0]:
            g = p.bt.read(key, R=ss.astype(np.uint64), R_mask=m, gc=True)
            if g["status"] == _abi.SS_LOG:
                p.from_log(key, pay.snapshot_time, True)
        p.ol.append(np.array([key], np.uint64), oc.reshape(1, len(oc)).astype(np.uint64),
                    oc_mask=m.reshape(1, 1), eff=np.array([eff], np.int64),
                    txid=np.array([txid], np.uint64))

    def read(self, key, R, rm):
        p = self.p
        g = p.bt.read(key, R=R.astype(np.uint64), R_mask=np.array([rm], np.uint64))
        if g["status"] == _abi.SS_LOG:
            p.log_reads += 1
            return p.from_log(key, vc(R, rm), False), g
        return ("ok", g["value"]), g


@pytest.mark.parametrize("d", [5, 8, 16, 64])
def test_counter_fused_vs_sequence_masked(eng, d):
    """Presence-masked counter partitions (the NIF's): entries with random DC
    sets (each holding its own DC), R missing DCs now and then.  Two
    partitions fed the same updates, one served by the fused read (k_read6,
    D = 16 / 64: k_read6w), one by the kernel sequence, both with the NIF's
    log fallback: every result field, the status and the ETS list sizes
    agree, and every served value equals the reference transcription's (its
    disk log serving what no cached snapshot does)."""
    import os
    K, steps = 16, 2500
    w = Workload(71 + d, K, d)
    full = (1 << d) - 1
    vn = po.MaterializerVnode(disk_log=True)
    quirk = set()
    checked = compared = 0
    with OpLog(eng, _abi.COUNTER_PN, d, K, sparse=True) as la, \
            OpLog(eng, _abi.COUNTER_PN, d, K, sparse=True) as lb:
        old = os.environ.get("AGN_READ6")
        try:
            os.environ["AGN_READ6"] = "1"
            _lib.env_changed()
            ba = Batcher(la, max_batch=8, cached=True)
            os.environ["AGN_READ6"] = "0"
            _lib.env_changed()
            bb = Batcher(lb, max_batch=8, cached=True)
        finally:
            if old is None:
                os.environ.pop("AGN_READ6", None)
            else:
                os.environ["AGN_READ6"] = old
            _lib.env_changed()
        with ba, bb:
            pa, pb = CounterNifPartition(la, ba, d), CounterNifPartition(lb, bb, d)
            for s in range(steps):
                key = int(w.rng.integers(0, K))
                if w.rng.random() < 0.7:
                    c, ss, ct, oc, eff = w.op(key)
                    mask = (rand_mask(w.rng, d) if w.rng.random() < 0.5 else full) | (1 << c)
                    pay = po.Payload(key, po.COUNTER_PN, eff, vc(ss, mask), (c, ct), s + 1)
                    try:
                        vn.update(key, pay)
                    except po.BadMatch:
                        quirk.add(key)
                    for p in (pa, pb):
                        p.update(key, pay, ss, oc, eff, s + 1, mask)
                    if has_placeholder(vn, key):
                        quirk.add(key)
                else:
                    R = w.read_clock(lag=400 if w.rng.random() < 0.85 else 20000)
                    rm = full if w.rng.random() < 0.8 else rand_mask(w.rng, d) | 1
                    (ra, ga), (rb, gb) = (p.read(key, R, rm) for p in (pa, pb))
                    for f in ("status", "value", "hole", "count", "flags", "err_pos"):
                        assert ga[f] == gb[f], (s, key, f, ga[f], gb[f])
                    assert np.array_equal(ga["lastct"], gb["lastct"]), (s, key)
                    assert np.array_equal(ga["lastct_mask"], gb["lastct_mask"]), (s, key)
                    assert ra == rb, (s, key)
                    compared += 1
                    if key in quirk:
                        continue
                    try:
                        want = vn.read(key, po.COUNTER_PN, vc(R, rm), po.IGNORE)
                    except po.BadMatch:
                        quirk.add(key)
                        continue
                    assert want == ra, (s, key, ga["status"], want, ra)
                    checked += 1
                    if has_placeholder(vn, key):
                        quirk.add(key)
            print(f"compared={compared} checked={checked} log_reads={pa.p.log_reads} "
                  f"log_gc={pa.p.log_gc} quirk={len(quirk)}/{K}")
            assert compared > 500 and checked > 400, (compared, checked)
            assert len(quirk) <= K // 4
            for a, b in zip(la.key_meta(), lb.key_meta()):
                assert np.array_equal(a, b)
            ln, ll, ct = la.key_meta()
    for k in range(K):
        if k in quirk or k not in vn.ops_cache:
            continue
        length, list_len = vn.ops_cache[k][1]
        assert (int(ln[k]), int(ll[k])) == (length, list_len), k
