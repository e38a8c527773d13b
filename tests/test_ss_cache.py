"""the materializer_vnode snapshot cache on device.

agn_ss_lookup = get_from_snapshot_cache/5 (+ vector_orddict:get_smaller/2,
including the store of the empty snapshot for an absent key) and
agn_ss_store = the cache half of materialize_snapshot/7 + internal_store_ss/5
+ insert_bigger/3 + snapshot_insert_gc/4 (src/materializer_vnode.erl:341-563).

The C oracle is checked against a literal dict restatement built on
oracle/py_oracle.py's VectorOrddict / vc_min; the GPU against the C oracle."""
import ctypes as C

import numpy as np
import pytest

from antidote_amd import _abi
from oracle import py_oracle as po
from antidote_amd.encode import alloc_result, log_struct, result_struct
from synth import compare, random_case

S = 10  # slots


def ptr(a):
    return None if a is None else a.ctypes.data


class Case:
    """A random cache, a batch of reads on distinct keys and the fields of the
    materialize result the store consumes."""

    def __init__(self, seed, K, D, sparse, n_req=None):
        rng = np.random.default_rng(seed)
        W = (D + 63) // 64
        self.K, self.D, self.W, self.sparse = K, D, W, sparse
        self.n = rng.integers(0, S, K).astype(np.uint32)  # 0..9 entries
        self.clock = np.zeros((K, S, D), np.uint64)
        self.mask = np.zeros((K, S, W), np.uint64) if sparse else None
        self.last_op = np.zeros((K, S), np.int64)
        self.value = rng.integers(-1000, 1000, (K, S)).astype(np.int64)
        for k in range(K):
            top = 1000 + rng.integers(0, 50, D)
            lop = int(rng.integers(40, 80))
            for j in range(int(self.n[k])):  # newest first: clocks decrease
                self.clock[k, j] = top - j * rng.integers(0, 20, D)
                self.last_op[k, j] = lop - 6 * j
                if sparse:
                    self.mask[k, j] = self._rand_mask(rng, 0.2)
        nr = n_req or K
        self.keys = rng.permutation(K)[:nr].astype(np.uint64)
        self.R = np.zeros((nr, D), np.uint64)
        for i, k in enumerate(self.keys):
            j = int(rng.integers(0, max(int(self.n[k]), 1) + 1))
            src = self.clock[k, min(j, S - 1)]
            self.R[i] = src + rng.integers(-3, 6, D)
        self.Rm = np.stack([self._rand_mask(rng, 0.05) for _ in range(nr)]) if sparse else None
        # materialize results for the store
        self.key_off = np.zeros(K + 1, np.uint64)
        self.key_off[1:] = np.cumsum(rng.integers(0, 3, K) * (rng.random(K) > 0.1))
        fl = np.zeros(nr, np.uint32)
        fl[rng.random(nr) < 0.8] |= _abi.F_NEWSS
        fl[rng.random(nr) < 0.05] |= _abi.F_CT_IGNORE
        fl[rng.random(nr) < 0.03] |= _abi.F_ERR_UNEXPECTED
        self.flags = fl
        self.count = rng.integers(0, 12, nr).astype(np.uint32)
        self.hole = np.array([int(self.last_op[k, 0]) + int(rng.integers(-2, 12))
                              for k in self.keys], np.int64)
        self.res_value = rng.integers(-10 ** 6, 10 ** 6, nr).astype(np.int64)
        self.lastct = np.zeros((nr, D), np.uint64)
        for i, k in enumerate(self.keys):
            self.lastct[i] = self.clock[k, 0] + rng.integers(-5, 30, D)
        self.lastct_mask = (np.stack([self._rand_mask(rng, 0.1) for _ in range(nr)])
                            if sparse else None)
        self.gc = (rng.random(nr) < 0.15).astype(np.uint8)

    def _rand_mask(self, rng, p_absent):
        m = np.zeros(self.W, np.uint64)
        for d in range(self.D):
            if rng.random() >= p_absent:
                m[d >> 6] |= np.uint64(1 << (d & 63))
        return m

    def cache_struct(self, arrs):
        c = _abi.AgnSsCache()
        c.n_dcs, c.slots, c.n_keys = self.D, S, self.K
        c.n, c.clock, c.last_op, c.value = (ptr(arrs[x]) for x in ("n", "clock", "last_op",
                                                                    "value"))
        c.clock_mask = ptr(arrs.get("mask"))
        return c

    def arrays(self):
        a = {"n": self.n.copy(), "clock": self.clock.copy(), "last_op": self.last_op.copy(),
             "value": self.value.copy()}
        if self.sparse:
            a["mask"] = self.mask.copy()
        return a


def run_oracle(lib, cs):
    a = cs.arrays()
    c = cs.cache_struct(a)
    nr, D, W = len(cs.keys), cs.D, cs.W
    out = {"sct": np.zeros((nr, D), np.uint64), "sctm": np.zeros((nr, W), np.uint64),
           "ign": np.zeros(nr, np.uint8), "base": np.zeros(nr, np.int64),
           "first": np.zeros(nr, np.uint8), "status": np.zeros(nr, np.uint8)}
    assert lib.oracle_ss_lookup(C.byref(c), nr, ptr(cs.keys), ptr(cs.R), ptr(cs.Rm),
                                ptr(out["sct"]), ptr(out["sctm"]) if cs.sparse else None,
                                ptr(out["ign"]), ptr(out["base"]), ptr(out["first"]),
                                ptr(out["status"])) == 0
    log = _abi.AgnLog()
    log.n_keys, log.n_dcs, log.key_off = cs.K, D, ptr(cs.key_off)
    res = _abi.AgnResult()
    res.value, res.hole, res.lastct = ptr(cs.res_value), ptr(cs.hole), ptr(cs.lastct)
    res.lastct_mask, res.count, res.flags = ptr(cs.lastct_mask), ptr(cs.count), ptr(cs.flags)
    out["prune"] = np.zeros(cs.K, np.uint8)
    out["thr"] = np.zeros((cs.K, D), np.uint64)
    out["thrm"] = np.zeros((cs.K, W), np.uint64)
    assert lib.oracle_ss_store(C.byref(c), C.byref(log), nr, ptr(cs.keys), ptr(out["first"]),
                               ptr(out["status"]), ptr(cs.gc), C.byref(res), None,
                               ptr(out["prune"]), ptr(out["thr"]),
                               ptr(out["thrm"]) if cs.sparse else None) == 0
    return a, out


# ------------------------------------------------------------------ dict restatement
def vc(row, mrow, D):
    return {d: int(row[d]) for d in range(D)
            if mrow is None or (int(mrow[d >> 6]) >> (d & 63)) & 1}


def py_model(cs):
    """Literal per-request walk of the Erlang with po.VectorOrddict."""
    D = cs.D
    caches = {}
    for k in range(cs.K):
        if cs.n[k]:
            caches[k] = po.VectorOrddict(
                [(vc(cs.clock[k, j], None if cs.mask is None else cs.mask[k, j], D),
                  (int(cs.last_op[k, j]), int(cs.value[k, j]))) for j in range(int(cs.n[k]))])
    looked, pruned = [], {}
    for i, k in enumerate(cs.keys):
        k = int(k)
        R = vc(cs.R[i], None if cs.Rm is None else cs.Rm[i], D)
        if k not in caches:
            caches[k] = po.VectorOrddict([({}, (0, 0))])
            looked.append(("new", None, 0, True))
            continue
        found, is_first = caches[k].get_smaller(R)
        looked.append(("hit" if found else "log", found[0] if found else None,
                       found[1][1] if found else 0, bool(found) and is_first))
    for i, k in enumerate(cs.keys):
        k = int(k)
        status, _sct, _base, is_first = looked[i]
        if status == "log" or cs.key_off[k + 1] == cs.key_off[k]:
            continue
        fl = int(cs.flags[i])
        if fl & (_abi.F_ERR_UNEXPECTED | _abi.F_ERR_CORRUPTED | _abi.F_ERR_CAPACITY):
            continue
        if fl & _abi.F_CT_IGNORE:
            continue
        gc = bool(cs.gc[i])
        refresh = bool(fl & _abi.F_NEWSS) and is_first and int(cs.count[i]) >= 5
        if not (refresh or gc):
            continue
        sd = caches[k]
        snap = (int(cs.hole[i]), int(cs.res_value[i]))
        should_insert = sd.size() == 0 or snap[0] - sd.first()[1][0] >= 5
        if not (should_insert or gc):
            continue
        ct = vc(cs.lastct[i], None if cs.lastct_mask is None else cs.lastct_mask[i], D)
        sd1 = sd.insert_bigger(ct, snap)
        if sd1.size() >= 10 or gc:
            p = sd1.sublist(1, 3)
            t, _ = p.last()
            for c1, _ in p.lst:
                t = po.vc_min([c1, t])
            pruned[k] = t
            caches[k] = p
        else:
            caches[k] = sd1
    return caches, looked, pruned


@pytest.mark.parametrize("D,sparse", [(1, False), (3, True), (8, False), (20, True),
                                      (70, True)])
def test_oracle_cache_vs_dict_restatement(oracle_lib, D, sparse):
    cs = Case(100 + D + sparse, 300, D, sparse)
    a, out = run_oracle(oracle_lib, cs)
    caches, looked, pruned = py_model(cs)
    W = cs.W
    for i, k in enumerate(cs.keys):
        st, sct, base, first = looked[i]
        assert out["status"][i] == {"hit": _abi.SS_HIT, "new": _abi.SS_NEW, "log": _abi.SS_LOG}[st]
        assert bool(out["first"][i]) == first
        assert int(out["base"][i]) == base
        if st == "hit":
            got = vc(out["sct"][i], out["sctm"][i] if sparse else None, D)
            assert got == ({d: v for d, v in sct.items()} if sparse else
                           {d: sct.get(d, 0) for d in range(D)})
    for k in range(cs.K):
        lst = caches.get(k, po.VectorOrddict())
        assert int(a["n"][k]) == lst.size(), k
        for j, (c, (lop, val)) in enumerate(lst.lst):
            got = vc(a["clock"][k, j], a["mask"][k, j] if sparse else None, D)
            want = c if sparse else {d: c.get(d, 0) for d in range(D)}
            assert got == want and int(a["last_op"][k, j]) == lop and int(a["value"][k, j]) == val
        assert bool(out["prune"][k]) == (k in pruned)
        if k in pruned:
            got = vc(out["thr"][k], out["thrm"][k] if sparse else None, D)
            want = pruned[k] if sparse else {d: pruned[k].get(d, 0) for d in range(D)}
            assert got == want
    assert out["prune"].any() and (out["status"] == _abi.SS_LOG).any()
    assert (out["status"] == _abi.SS_HIT).any() and (out["status"] == _abi.SS_NEW).any()
    _ = W


@pytest.mark.gpu
@pytest.mark.parametrize("D,sparse,K", [(3, True, 20000), (8, False, 200000), (16, False, 50000),
                                        (64, True, 20000), (130, True, 5000)])
def test_cache_gpu_vs_oracle(eng, oracle_lib, D, sparse, K):
    cs = Case(7 * D + K, K, D, sparse, n_req=K // 2)
    want_a, want = run_oracle(oracle_lib, cs)
    nr, W = len(cs.keys), cs.W
    a = cs.arrays()
    dev = {n: eng.upload(x) for n, x in a.items()}
    c = _abi.AgnSsCache()
    c.n_dcs, c.slots, c.n_keys = D, S, cs.K
    c.n, c.clock, c.last_op, c.value = (dev[x].ptr for x in ("n", "clock", "last_op", "value"))
    c.clock_mask = dev["mask"].ptr if sparse else None
    up = lambda x: eng.upload(x) if x is not None else None  # noqa: E731
    keys, R, Rm = up(cs.keys), up(cs.R), up(cs.Rm)
    o = {"sct": eng.empty(nr * D * 8), "sctm": eng.empty(nr * W * 8), "ign": eng.empty(nr),
         "base": eng.empty(nr * 8), "first": eng.empty(nr), "status": eng.empty(nr)}
    eng.ss_lookup(c, nr, keys.ptr, R.ptr, Rm.ptr if Rm else None, o["sct"].ptr,
                  o["sctm"].ptr if sparse else None, o["ign"].ptr, o["base"].ptr,
                  o["first"].ptr, o["status"].ptr)
    got = {"status": eng.download(o["status"], np.uint8, (nr,)),
           "first": eng.download(o["first"], np.uint8, (nr,)),
           "base": eng.download(o["base"], np.int64, (nr,)),
           "ign": eng.download(o["ign"], np.uint8, (nr,)),
           "sct": eng.download(o["sct"], np.uint64, (nr, D))}
    for n in ("status", "first", "base", "ign"):
        assert np.array_equal(got[n], want[n]), n
    hit = want["status"] == _abi.SS_HIT
    assert np.array_equal(got["sct"][hit], want["sct"][hit])
    if sparse:
        gm = eng.download(o["sctm"], np.uint64, (nr, W))
        assert np.array_equal(gm[hit], want["sctm"][hit])
    # store
    log = _abi.AgnLog()
    log.n_keys, log.n_dcs = cs.K, D
    ko = up(cs.key_off)
    log.key_off = ko.ptr
    res = _abi.AgnResult()
    rb = {n: up(getattr(cs, n)) for n in ("res_value", "hole", "lastct", "lastct_mask", "count",
                                          "flags")}
    res.value, res.hole, res.lastct = rb["res_value"].ptr, rb["hole"].ptr, rb["lastct"].ptr
    res.lastct_mask = rb["lastct_mask"].ptr if sparse else None
    res.count, res.flags = rb["count"].ptr, rb["flags"].ptr
    gcb = up(cs.gc)
    pr, th, thm = eng.empty(cs.K), eng.empty(cs.K * D * 8), eng.empty(cs.K * W * 8)
    eng.ss_store(c, log, nr, keys.ptr, o["first"].ptr, o["status"].ptr, gcb.ptr, res, None,
                 pr.ptr, th.ptr, thm.ptr if sparse else None)
    gp = eng.download(pr, np.uint8, (cs.K,))
    assert np.array_equal(gp, want["prune"])
    sel = want["prune"] == 1
    assert np.array_equal(eng.download(th, np.uint64, (cs.K, D))[sel], want["thr"][sel])
    if sparse:
        assert np.array_equal(eng.download(thm, np.uint64, (cs.K, W))[sel], want["thrm"][sel])
    gn = eng.download(dev["n"], np.uint32, (cs.K,))
    assert np.array_equal(gn, want_a["n"])
    for name, dt, shape in (("clock", np.uint64, (cs.K, S, D)), ("last_op", np.int64, (cs.K, S)),
                            ("value", np.int64, (cs.K, S))) + \
            ((("mask", np.uint64, (cs.K, S, W)),) if sparse else ()):
        g = eng.download(dev[name], dt, shape)
        for k in np.nonzero(gn)[0][:5000]:
            assert np.array_equal(g[k, :gn[k]], want_a[name][k, :gn[k]]), (name, k)


@pytest.mark.gpu
@pytest.mark.parametrize("split,np_", [("0", "1"), ("0", "2"), ("1", "")],
                         ids=["fused", "fused_pair", "batched"])
@pytest.mark.parametrize("D", [1, 3, 5, 8])
def test_read_cached_vs_sequence(eng, monkeypatch, D, split, np_):
    """agn_read_cached (read/6 in one kernel: lookup -> materialize from the
    cached base -> store policy) equals agn_ss_lookup -> agn_materialize ->
    agn_ss_store on two caches that start empty: every result field, the
    lookup status, the prune flags (per request vs per key), the GC
    thresholds and the cache contents, over rounds of batches on distinct
    keys with GC reads mixed in (cold reads, hits, stores, prunes).  split =
    "0": the fused kernel, one request per wave or two (AGN_READ6_NP; the
    odd batch sizes leave the last wave one request); "1": agn_read_cached's
    bulk form (the batched kernels with per-request prune flags,
    AGN_READ_CACHED_SPLIT=1)."""
    monkeypatch.setenv("AGN_READ_CACHED_SPLIT", split)
    monkeypatch.setenv("AGN_READ6_NP", np_)
    K = 3000
    # 0..150 ops per key: one, two and three 64-op chunks
    log, req, _ = random_case(501 + D, _abi.COUNTER_PN, K, D, 150, txid=0.2, empty=0.05)
    rng = np.random.default_rng(D)
    dlog = eng.upload_log(log)
    dlog.struct.oc_mask = None

    def cache():
        bufs = {"n": eng.upload(np.zeros(K, np.uint32)),
                "clock": eng.empty(8 * K * S * D), "last_op": eng.empty(8 * K * S),
                "value": eng.empty(8 * K * S)}
        c = _abi.AgnSsCache()
        c.n_dcs, c.slots, c.n_keys = D, S, K
        c.n, c.clock, c.last_op, c.value = (bufs[x].ptr for x in ("n", "clock", "last_op", "value"))
        c.clock_mask = None
        return c, bufs

    ca, ba = cache()
    cb, bb = cache()
    for rnd in range(4):
        nr = 1501 + 300 * rnd
        keys = rng.permutation(K)[:nr].astype(np.uint64)
        R = req.R[keys.astype(np.int64)] + rng.integers(0, 3, (nr, D)).astype(np.uint64)
        tx = req.txid[keys.astype(np.int64)].copy()
        gc = (rng.random(nr) < 0.2).astype(np.uint8)
        dk, dR, dtx, dgc = (eng.upload(x) for x in (keys, np.ascontiguousarray(R), tx, gc))
        # the sequence
        o = {"sct": eng.empty(nr * D * 8), "ign": eng.empty(nr), "base": eng.empty(nr * 8),
             "first": eng.empty(nr), "status": eng.empty(nr), "prune": eng.empty(K),
             "thr": eng.empty(K * D * 8)}
        eng.ss_lookup(ca, nr, dk.ptr, dR.ptr, None, o["sct"].ptr, None, o["ign"].ptr,
                      o["base"].ptr, o["first"].ptr, o["status"].ptr)
        rs = _abi.AgnRead()
        rs.n_dcs, rs.req_type, rs.n_req = D, _abi.COUNTER_PN, nr
        rs.keys, rs.R, rs.txid = dk.ptr, dR.ptr, dtx.ptr
        rs.sct, rs.sct_ignore, rs.base_value = o["sct"].ptr, o["ign"].ptr, o["base"].ptr
        res_a = eng.alloc_result(nr, D, sparse=False)
        eng.materialize(dlog, rs, res_a)
        eng.ss_store(ca, dlog, nr, dk.ptr, o["first"].ptr, o["status"].ptr, dgc.ptr, res_a, None,
                     o["prune"].ptr, o["thr"].ptr, None)
        # fused
        res_b = eng.alloc_result(nr, D, sparse=False)
        st_b, pr_b, thr_b = eng.empty(nr), eng.empty(nr), eng.empty(K * D * 8)
        eng.read_cached(cb, dlog, nr, dk.ptr, dR.ptr, dtx.ptr, dgc.ptr, res_b, st_b.ptr, pr_b.ptr,
                        thr_b.ptr)
        eng.sync()
        ga, gb = eng.fetch_result(res_a), eng.fetch_result(res_b)
        for f in ("value", "hole", "lastct", "count", "flags", "err_pos"):
            assert np.array_equal(getattr(ga, f), getattr(gb, f)), (rnd, f)
        sa = eng.download(o["status"], np.uint8, (nr,))
        assert np.array_equal(sa, eng.download(st_b, np.uint8, (nr,))), rnd
        pa = eng.download(o["prune"], np.uint8, (K,))[keys.astype(np.int64)]
        pb = eng.download(pr_b, np.uint8, (nr,))
        assert np.array_equal(pa, pb), rnd
        sel = keys[pa == 1].astype(np.int64)
        assert np.array_equal(eng.download(o["thr"], np.uint64, (K, D))[sel],
                              eng.download(thr_b, np.uint64, (K, D))[sel]), rnd
        na = eng.download(ba["n"], np.uint32, (K,))
        assert np.array_equal(na, eng.download(bb["n"], np.uint32, (K,))), rnd
        for name, dt, shape in (("clock", np.uint64, (K, S, D)), ("last_op", np.int64, (K, S)),
                                ("value", np.int64, (K, S))):
            xa, xb = eng.download(ba[name], dt, shape), eng.download(bb[name], dt, shape)
            for k in np.nonzero(na)[0]:
                assert np.array_equal(xa[k, :na[k]], xb[k, :na[k]]), (rnd, name, k)
        if rnd == 0:
            assert (sa == _abi.SS_NEW).all()
        else:
            assert (sa == _abi.SS_HIT).any()
        for b in list(o.values()) + [dk, dR, dtx, dgc, st_b, pr_b, thr_b] + \
                list(res_a.bufs.values()) + list(res_b.bufs.values()):
            b.free()


def oracle_read_cached(lib, hc, ls, keys, R, tx, gc, D):
    """read/6 for a batch through the C oracle on the host cache `hc`:
    oracle_ss_lookup -> oracle_materialize -> oracle_ss_store
    (materializer_vnode.erl:384-413, 466-509).  Returns (result, status,
    prune flags per key, thresholds per key)."""
    nr, K = len(keys), hc.n_keys
    sct, ign = np.zeros((nr, D), np.uint64), np.zeros(nr, np.uint8)
    base, first, status = np.zeros(nr, np.int64), np.zeros(nr, np.uint8), np.zeros(nr, np.uint8)
    assert lib.oracle_ss_lookup(C.byref(hc), nr, ptr(keys), ptr(R), None, ptr(sct), None,
                                ptr(ign), ptr(base), ptr(first), ptr(status)) == 0
    rq = _abi.AgnRead()
    rq.n_req, rq.keys, rq.R, rq.R_mask = nr, ptr(keys), ptr(R), None
    rq.sct, rq.sct_mask, rq.sct_ignore, rq.txid = ptr(sct), None, ptr(ign), ptr(tx)
    rq.req_type, rq.base_value = _abi.COUNTER_PN, ptr(base)
    res = alloc_result(nr, D, sparse=False)
    rs = result_struct(res)
    assert lib.oracle_materialize(C.byref(ls), C.byref(rq), C.byref(rs), 4) == 0
    prune, thr = np.zeros(K, np.uint8), np.zeros((K, D), np.uint64)
    assert lib.oracle_ss_store(C.byref(hc), C.byref(ls), nr, ptr(keys), ptr(first), ptr(status),
                               ptr(gc), C.byref(rs), None, ptr(prune), ptr(thr), None) == 0
    return res, status, prune, thr


@pytest.mark.gpu
def test_read_cached_default_dispatch(eng, oracle_lib, monkeypatch):
    """A bulk batch (33k requests, D = 8, keys of up to 64 ops: those past 32
    take the fused kernel's second chunk) through agn_read_cached's default
    dispatch (the fused k_read6: D = 8 switches only from 5M requests) and with
    the batched kernels forced (AGN_READ_CACHED_SPLIT=1), each against the C
    oracle's lookup -> materialize -> store chain on a host cache: outputs,
    status, prune flags, thresholds and the caches, over a cold round and two
    warm rounds with GC reads (the second with newly included ops)."""
    K, D, nr = 36_000, 8, 33_000
    log, req, _ = random_case(977, _abi.COUNTER_PN, K, D, 64, txid=0.2, empty=0.05)
    lens = np.diff(log.key_off.astype(np.int64))
    assert (lens > 32).mean() > 0.3
    dlog = eng.upload_log(log)
    dlog.struct.oc_mask = None
    ls = log_struct(log)
    ls.oc_mask = None
    rng = np.random.default_rng(5)
    hcache = {"n": np.zeros(K, np.uint32), "clock": np.zeros((K, S, D), np.uint64),
              "last_op": np.zeros((K, S), np.int64), "value": np.zeros((K, S), np.int64)}
    hc = _abi.AgnSsCache()
    hc.n_dcs, hc.slots, hc.n_keys = D, S, K
    hc.n, hc.clock, hc.last_op, hc.value = (ptr(hcache[x]) for x in ("n", "clock", "last_op",
                                                                     "value"))
    hc.clock_mask = None

    def cache():
        bufs = {"n": eng.upload(np.zeros(K, np.uint32)),
                "clock": eng.empty(8 * K * S * D), "last_op": eng.empty(8 * K * S),
                "value": eng.empty(8 * K * S)}
        c = _abi.AgnSsCache()
        c.n_dcs, c.slots, c.n_keys = D, S, K
        c.n, c.clock, c.last_op, c.value = (bufs[x].ptr for x in ("n", "clock", "last_op", "value"))
        c.clock_mask = None
        return c, bufs

    caches = [cache(), cache()]
    try:
        for rnd in range(3):
            keys = rng.permutation(K)[:nr].astype(np.uint64)
            ki = keys.astype(np.int64)
            R = np.ascontiguousarray(req.R[ki] + rng.integers(0, 3 if rnd < 2 else 40, (nr, D))
                                     .astype(np.uint64))
            tx = req.txid[ki].copy()
            gc = (rng.random(nr) < (0.0 if rnd == 0 else 0.2)).astype(np.uint8)
            want, wst, wpr, wthr = oracle_read_cached(oracle_lib, hc, ls, keys, R, tx, gc, D)
            dk, dR, dtx, dgc = (eng.upload(x) for x in (keys, R, tx, gc))
            for (c, bufs), split in zip(caches, (None, "1")):
                ctx = (rnd, split)
                if split is None:
                    monkeypatch.delenv("AGN_READ_CACHED_SPLIT", raising=False)
                else:
                    monkeypatch.setenv("AGN_READ_CACHED_SPLIT", split)
                res = eng.alloc_result(nr, D, sparse=False)
                st, pr, thr = eng.empty(nr), eng.empty(nr), eng.empty(K * D * 8)
                eng.lib.agn_memset_d(eng.ctx, thr.ptr, 0, K * D * 8, None)
                eng.read_cached(c, dlog, nr, dk.ptr, dR.ptr, dtx.ptr, dgc.ptr, res, st.ptr, pr.ptr,
                                thr.ptr)
                eng.sync()
                got = eng.fetch_result(res)
                bad = compare(_abi.COUNTER_PN, D, got, want, False, nr)
                assert not bad, (ctx, bad[:10])
                assert np.array_equal(eng.download(st, np.uint8, (nr,)), wst), ctx
                # read_cached flags per request, the store per key (keys distinct)
                gp = eng.download(pr, np.uint8, (nr,))
                assert np.array_equal(gp, wpr[ki]), ctx
                pk = ki[gp == 1]
                assert np.array_equal(eng.download(thr, np.uint64, (K, D))[pk], wthr[pk]), ctx
                n = eng.download(bufs["n"], np.uint32, (K,))
                assert np.array_equal(n, hcache["n"]), ctx
                live = np.arange(S)[None, :] < n[:, None]
                for name, dt, shape in (("clock", np.uint64, (K, S, D)),
                                        ("last_op", np.int64, (K, S)),
                                        ("value", np.int64, (K, S))):
                    x = eng.download(bufs[name], dt, shape)
                    assert np.array_equal(x[live], hcache[name][live]), (ctx, name)
                for b in [st, pr, thr] + list(res.bufs.values()):
                    b.free()
            if rnd >= 1:
                assert (wst == _abi.SS_HIT).any() and wpr.any()
            if rnd == 2:
                assert (want.count > 0).any()
            for b in (dk, dR, dtx, dgc):
                b.free()
    finally:
        for _c, bufs in caches:
            for b in bufs.values():
                b.free()
