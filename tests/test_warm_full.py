"""The warm read/6 paths bench.py times, at the bench's full sizes, against the
C oracle on a sampled key set (VERDICT r5 "do this" #2).

Reference path: materializer_vnode:read/6 -> internal_read/7 ->
get_from_snapshot_cache/5 -> materialize_snapshot/7 -> internal_store_ss/5
(src/materializer_vnode.erl:96-102, 371-413, 466-509).

The device runs every key of the configuration (the bench's own generator
seeds, so the very data the bench line measures); the oracle replays the same
rounds for each sampled key alone -- oracle_ss_lookup -> oracle_materialize ->
oracle_ss_store on a one-key cache, each key's log host-generated from the
same SplitMix64 streams.  Keys are independent in every step (distinct keys
per batch), so the one-key replay is the reference's answer for that key.
Rounds, as the bench runs them and past it:
  0  R = the generator's read clock, no GC reads   (priming: empty snapshot
     stored, cold materialize, store)
  1  the same R                                     (the timed steady state:
     every key a hit, materialize from the cached base)
  2  R + U[0, 4000) per DC, 10 % GC reads            (newly included ops, the
     store policy's insert / GC prune thresholds)
Compared per sampled key and round: value (or the set/register state),
NewLastOp, LastOpCt, Count, flags, err_pos, lookup status, prune flag,
GC threshold, and the key's cache slots (clock, last op id, value / state).
"""
import ctypes as C

import numpy as np
import pytest

from antidote_amd import _abi
from antidote_amd.encode import alloc_result, result_struct
from antidote_amd.engine import free_gen_host, gen_host, host_view

pytestmark = pytest.mark.gpu

S = _abi.SNAPSHOT_THRESHOLD
N_SAMPLE = 512

# bench.py CONFIGS 2, 3, 4 (N = 1), the bench's seeds
CFG2 = dict(crdt_type=1, n_dcs=8, n_keys=10_000_000, ops_per_key=64, n_elems=0,
            seed=20250112 + 1)
CFG3 = dict(crdt_type=2, n_dcs=16, n_keys=1_000_000, ops_per_key=256, n_elems=32,
            seed=20250112 + 2)
CFG4 = dict(crdt_type=3, n_dcs=64, n_keys=1_000_000, ops_per_key=100, n_elems=16,
            seed=20250112 + 3)


def p(a):
    return None if a is None else a.ctypes.data


class At:
    """A device address (for Engine.download of one slice)."""

    def __init__(self, ptr):
        self.ptr = ptr


def rows_at(eng, ptr, dtype, row, idx):
    """Rows idx of a device array of `row`-shaped rows, one copy per row."""
    isz = int(np.prod(row)) * np.dtype(dtype).itemsize
    return np.stack([eng.download(At(ptr + int(i) * isz), dtype, row) for i in idx])


def round_inputs(rnd, K, D, R0):
    """(R[K][D], gc[K] or None) of round rnd, from the generator's R0."""
    if rnd < 2:
        return R0, None
    rng = np.random.default_rng(777 + D)
    R = R0 + rng.integers(0, 4000, (K, D), dtype=np.uint64)
    gc = (rng.random(K) < 0.1).astype(np.uint8)
    return R, gc


class KeyReplay:
    """One key's read/6 rounds through the C oracle on a one-key cache.  For
    set_aw / register_mv the cached value is a handle into self.states (the
    snapshot's state: the reference caches the full #materialized_snapshot)."""

    def __init__(self, lib, spec, k):
        self.lib, self.D, self.tags = lib, spec["n_dcs"], spec["crdt_type"] != 1
        g = _abi.AgnGenCfg(crdt_type=spec["crdt_type"], n_dcs=self.D, n_keys=1,
                           ops_per_key=spec["ops_per_key"], n_elems=spec["n_elems"],
                           seed=spec["seed"], key_base=int(k), key_stride=1, warm=0)
        self.hl, self.hr = gen_host(g)
        self.N = spec["ops_per_key"]
        self.n = np.zeros(1, np.uint32)
        self.clock = np.zeros(S * self.D, np.uint64)
        self.last_op = np.zeros(S, np.int64)
        self.value = np.zeros(S, np.int64)
        self.states = {0: (np.zeros(0, np.uint32), np.zeros(0, np.uint64))}
        self.c = _abi.AgnSsCache()
        self.c.n_dcs, self.c.slots, self.c.n_keys = self.D, S, 1
        self.c.n, self.c.clock, self.c.last_op, self.c.value = (
            p(self.n), p(self.clock), p(self.last_op), p(self.value))
        self.c.clock_mask = None

    def close(self):
        free_gen_host(self.hl, self.hr)

    def R0(self):
        return host_view(self.hr.R, np.uint64, self.D).copy()

    def step(self, R, gc):
        D, lib = self.D, self.lib
        R = np.ascontiguousarray(R, np.uint64)
        sct, ign = np.zeros(D, np.uint64), np.zeros(4, np.uint8)
        base, first, status = np.zeros(1, np.int64), np.zeros(4, np.uint8), np.zeros(4, np.uint8)
        assert lib.oracle_ss_lookup(C.byref(self.c), 1, None, p(R), None, p(sct), None, p(ign),
                                    p(base), p(first), p(status)) == 0
        rq = _abi.AgnRead()
        C.memmove(C.addressof(rq), C.addressof(self.hr), C.sizeof(_abi.AgnRead))
        rq.n_req, rq.keys, rq.R, rq.R_mask = 1, None, p(R), None
        rq.sct, rq.sct_mask, rq.sct_ignore = p(sct), None, p(ign)
        cap = None
        if self.tags:
            btag, btok = self.states[int(base[0])]
            boff = np.array([0, len(btag)], np.uint64)
            # one spare element: a valid address for an empty state
            bt = np.append(np.ascontiguousarray(btag, np.uint32), np.uint32(0))
            bk = np.append(np.ascontiguousarray(btok, np.uint64), np.uint64(0))
            rq.base_value, rq.base_off = None, p(boff)
            rq.base_tag, rq.base_tok = p(bt), p(bk)
            cap = np.array([0, self.N + len(btag)], np.uint64)
        else:
            rq.base_value = p(base)
        res = alloc_result(1, D, sparse=False, cap_off=cap)
        rs = result_struct(res)
        assert lib.oracle_materialize(C.byref(self.hl), C.byref(rq), C.byref(rs), 1) == 0
        handle = None
        if self.tags:
            h = len(self.states)
            nn = int(res.out_n[0])
            self.states[h] = (res.out_tag[:nn].copy(), res.out_tok[:nn].copy())
            handle = np.array([h], np.int64)
        prune, thr = np.zeros(4, np.uint8), np.zeros(D, np.uint64)
        gcv = np.array([gc, 0, 0, 0], np.uint8)
        assert lib.oracle_ss_store(C.byref(self.c), C.byref(self.hl), 1, None, p(first),
                                   p(status), p(gcv), C.byref(rs), p(handle), p(prune), p(thr),
                                   None) == 0
        return {"res": res, "status": int(status[0]), "prune": int(prune[0]), "thr": thr}

    def state_of(self, slot):
        return self.states[int(self.value[slot])]


def sample_keys(K, seed):
    rng = np.random.default_rng(seed)
    s = np.sort(rng.choice(K, N_SAMPLE, replace=False))
    s[0], s[-1] = 0, K - 1
    return s


class DevCache:
    """A device snapshot cache over every key of the log (+ a state arena for
    set_aw / register_mv, sized as bench.warm_bench_tags sizes it)."""

    def __init__(self, eng, K, D, N, tags):
        self.eng, self.K, self.D = eng, K, D
        self.bufs = {"n": eng.empty(4 * K), "clock": eng.empty(8 * K * S * D),
                     "last_op": eng.empty(8 * K * S), "value": eng.empty(8 * K * S)}
        eng.lib.agn_memset_d(eng.ctx, self.bufs["n"].ptr, 0, 4 * K, None)
        c = _abi.AgnSsCache()
        c.n_dcs, c.slots, c.n_keys = D, S, K
        c.n, c.clock, c.last_op, c.value = (self.bufs[x].ptr
                                            for x in ("n", "clock", "last_op", "value"))
        c.clock_mask = None
        if tags:
            cap = 3 * K * N
            self.bufs.update(ctl=eng.empty(32), st_tag=eng.empty(4 * cap),
                             st_tok=eng.empty(8 * cap))
            eng.lib.agn_memset_d(eng.ctx, self.bufs["ctl"].ptr, 0, 32, None)
            c.state_tag, c.state_tok = self.bufs["st_tag"].ptr, self.bufs["st_tok"].ptr
            c.state_cap, c.state_ctl = cap, self.bufs["ctl"].ptr
        self.c = c

    def rows(self, sample):
        """(n, clock, last_op, value) of the sampled keys."""
        e, D, b = self.eng, self.D, self.bufs
        n = rows_at(e, b["n"].ptr, np.uint32, (1,), sample)[:, 0]
        clock = rows_at(e, b["clock"].ptr, np.uint64, (S, D), sample)
        lop = rows_at(e, b["last_op"].ptr, np.int64, (S,), sample)
        val = rows_at(e, b["value"].ptr, np.int64, (S,), sample)
        return n, clock, lop, val

    def state(self, ref):
        """The (tags, tokens) of an AGN_SS_STATE reference in the arena."""
        start, pairs = _abi.ss_state_unpack(int(ref))
        ctl = self.eng.download(self.bufs["ctl"], np.uint64, (4,))
        assert int(ctl[2]) == 0 and start + pairs <= int(ctl[0]), "state arena"
        if pairs == 0:
            return np.zeros(0, np.uint32), np.zeros(0, np.uint64)
        tg = self.eng.download(At(self.bufs["st_tag"].ptr + 4 * start), np.uint32, (pairs,))
        tk = self.eng.download(At(self.bufs["st_tok"].ptr + 8 * start), np.uint64, (pairs,))
        return tg, tk

    def free(self):
        for b in self.bufs.values():
            b.free()


def sampled_result(eng, res, sample, D, tags):
    """The result fields of the sampled requests (+ each one's state)."""
    b = res.bufs
    out = {"value": rows_at(eng, b["value"].ptr, np.int64, (1,), sample)[:, 0],
           "hole": rows_at(eng, b["hole"].ptr, np.int64, (1,), sample)[:, 0],
           "lastct": rows_at(eng, b["lastct"].ptr, np.uint64, (D,), sample),
           "count": rows_at(eng, b["count"].ptr, np.uint32, (1,), sample)[:, 0],
           "flags": rows_at(eng, b["flags"].ptr, np.uint32, (1,), sample)[:, 0],
           "err_pos": rows_at(eng, b["err_pos"].ptr, np.uint32, (1,), sample)[:, 0]}
    if tags:
        off = rows_at(eng, b["out_off"].ptr, np.uint64, (1,), sample)[:, 0]
        nn = rows_at(eng, b["out_n"].ptr, np.uint32, (1,), sample)[:, 0]
        out["state"] = [
            (eng.download(At(b["out_tag"].ptr + 4 * int(o)), np.uint32, (int(n),)),
             eng.download(At(b["out_tok"].ptr + 8 * int(o)), np.uint64, (int(n),)))
            for o, n in zip(off, nn)]
    return out


def check_round(rnd, sample, reps, got, want, dev, tags):
    res, status, prune, thr = got
    n, clock, lop, val = dev.rows(sample)
    for j, k in enumerate(sample):
        w, r = want[j], reps[j]
        wr = w["res"]
        ctx = (rnd, int(k))
        assert int(status[j]) == w["status"], ctx
        assert int(res["flags"][j]) == int(wr.flags[0]), ctx
        assert int(res["hole"][j]) == int(wr.hole[0]), ctx
        assert int(res["count"][j]) == int(wr.count[0]), ctx
        assert int(res["err_pos"][j]) == int(wr.err_pos[0]), ctx
        assert np.array_equal(res["lastct"][j], wr.lastct[0]), ctx
        if tags:
            nn = int(wr.out_n[0])
            gt, gk = res["state"][j]
            assert len(gt) == nn, ctx
            assert np.array_equal(gt, wr.out_tag[:nn]), ctx
            assert np.array_equal(gk, wr.out_tok[:nn]), ctx
        else:
            assert int(res["value"][j]) == int(wr.value[0]), ctx
        assert int(prune[j]) == w["prune"], ctx
        if w["prune"]:
            assert np.array_equal(thr[j], w["thr"]), ctx
        # the key's cache slots
        m = int(r.n[0])
        assert int(n[j]) == m, ctx
        assert np.array_equal(clock[j, :m], r.clock.reshape(S, -1)[:m]), ctx
        assert np.array_equal(lop[j, :m], r.last_op[:m]), ctx
        for s in range(m):
            if tags:
                gt, gk = dev.state(val[j, s])
                wt, wk = r.state_of(s)
                assert np.array_equal(gt, wt) and np.array_equal(gk, wk), (ctx, s)
            else:
                assert int(val[j, s]) == int(r.value[s]), (ctx, s)


def run_rounds(eng, oracle_lib, spec, forms):
    """forms[rnd] = "read_cached" (agn_read_cached, default dispatch) or
    "sequence" (agn_ss_lookup -> agn_materialize -> agn_ss_store, the calls
    bench.warm_bench times) per round."""
    cfg = _abi.AgnGenCfg(key_base=0, key_stride=1, warm=0, **spec)
    K, D, N = cfg.n_keys, cfg.n_dcs, cfg.ops_per_key
    tags = cfg.crdt_type != 1
    dl, dr = eng.gen_dev(cfg)
    dev = DevCache(eng, K, D, N, tags)
    sample = sample_keys(K, cfg.seed)
    reps = [KeyReplay(oracle_lib, spec, k) for k in sample]
    cap = np.arange(K + 1, dtype=np.uint64) * np.uint64(N) if tags else None
    res = eng.alloc_result(K, D, sparse=False, cap_off=cap)
    keys = eng.upload(np.arange(K, dtype=np.uint64))
    R0 = eng.download(At(dr.R), np.uint64, (K, D))
    for j, k in enumerate(sample):
        assert np.array_equal(reps[j].R0(), R0[k])  # same generator streams
    seq = {n: eng.empty(sz) for n, sz in (("sct", 8 * K * D), ("ign", K), ("base", 8 * K),
                                          ("first", K), ("status", K), ("prune", K),
                                          ("thr", 8 * K * D))}
    tmp = []
    try:
        for rnd, form in enumerate(forms):
            R, gc = round_inputs(rnd, K, D, R0)
            dR = eng.upload(np.ascontiguousarray(R))
            dgc = eng.upload(gc) if gc is not None else None
            tmp += [dR] + ([dgc] if dgc else [])
            eng.lib.agn_memset_d(eng.ctx, seq["thr"].ptr, 0, 8 * K * D, None)
            if form == "read_cached":
                eng.read_cached(dev.c, dl, K, keys.ptr, dR.ptr, dr.txid,
                                dgc.ptr if dgc else None, res, seq["status"].ptr,
                                seq["prune"].ptr, seq["thr"].ptr)
                eng.sync()
                prune = rows_at(eng, seq["prune"].ptr, np.uint8, (1,), sample)[:, 0]
            else:
                eng.ss_lookup(dev.c, K, None, dR.ptr, None, seq["sct"].ptr, None, seq["ign"].ptr,
                              seq["base"].ptr, seq["first"].ptr, seq["status"].ptr)
                rq = _abi.AgnRead()
                C.memmove(C.addressof(rq), C.addressof(dr), C.sizeof(_abi.AgnRead))
                rq.R = dR.ptr
                rq.sct, rq.sct_ignore, rq.base_value = seq["sct"].ptr, seq["ign"].ptr, \
                    seq["base"].ptr
                if tags:
                    rq.base_off, rq.base_tag, rq.base_tok = None, dev.c.state_tag, \
                        dev.c.state_tok
                eng.materialize(dl, rq, res)
                eng.ss_store(dev.c, dl, K, None, seq["first"].ptr, seq["status"].ptr,
                             dgc.ptr if dgc else None, res, None, seq["prune"].ptr,
                             seq["thr"].ptr, None)
                eng.sync()
                # agn_ss_store's prune flags are per key (identity keys here)
                prune = rows_at(eng, seq["prune"].ptr, np.uint8, (1,), sample)[:, 0]
            status_all = eng.download(seq["status"], np.uint8, (K,))
            status = status_all[sample]
            thr = rows_at(eng, seq["thr"].ptr, np.uint64, (D,), sample)
            got = (sampled_result(eng, res, sample, D, tags), status, prune, thr)
            want = [r.step(R[k], 0 if gc is None else int(gc[k])) for r, k in zip(reps, sample)]
            check_round(rnd, sample, reps, got, want, dev, tags)
            # the bench's shape: every key a hit from round 1 on
            if rnd == 1:
                assert (status_all == _abi.SS_HIT).all()
            if rnd == 2:
                assert any(w["prune"] for w in want) and \
                    any(int(w["res"].count[0]) for w in want)
    finally:
        for r in reps:
            r.close()
        for b in list(seq.values()) + tmp + [keys] + list(res.bufs.values()):
            b.free()
        dev.free()
        eng.free_gen(dl, dr)


@pytest.mark.parametrize("split", ["0", None], ids=["fused", "default"])
def test_warm_cfg2_read_cached_full_size(eng, oracle_lib, monkeypatch, split):
    """cfg2_warm: 10M keys x 64 ops, D = 8, agn_read_cached for all three
    rounds: the fused k_read6 forced (AGN_READ_CACHED_SPLIT=0: lookup -> warm
    materialize over two 32-op chunks -> store in one launch) and the default
    dispatch, which at 10M requests runs the batched kernels."""
    if split is None:
        monkeypatch.delenv("AGN_READ_CACHED_SPLIT", raising=False)
    else:
        monkeypatch.setenv("AGN_READ_CACHED_SPLIT", split)
    run_rounds(eng, oracle_lib, CFG2, ["read_cached"] * 3)


def test_warm_cfg2_sequence_full_size(eng, oracle_lib):
    """cfg2_warm's materialize leg (the bench's roofline kernel): lookup ->
    agn_materialize from the cached base -> store, all three rounds."""
    run_rounds(eng, oracle_lib, CFG2, ["sequence"] * 3)


@pytest.mark.parametrize("spec", [CFG3, CFG4], ids=["cfg3_set_aw", "cfg4_register_mv"])
def test_warm_tags_full_size(eng, oracle_lib, spec):
    """cfg3_warm / cfg4_warm: the state-arena path at 1M keys (k_tags reading
    each hit's base state from the arena) through the sequence the bench
    times, then agn_read_cached (the batched kernels) for the GC round."""
    run_rounds(eng, oracle_lib, spec, ["sequence", "sequence", "read_cached"])
