"""the log-read fallback and the recovery ingest —
logging_vnode get_ops_from_log / filter_terms_for_key / handle_commit
(src/logging_vnode.erl:522-549, 660-779) over a decoded partition log,
producing the device op log (get_up_to_time's #snapshot_get_response{} ops,
reverse_and_add_op_id ids; load_from_log's op_insert_gc ids).

The C oracle is checked against a literal dict transcription of the Erlang
walk below; the GPU hash-join + stable-sort implementation against the C
oracle on every output array."""
import ctypes as C

import numpy as np
import pytest

from antidote_amd import _abi
from oracle import py_oracle as po


def ptr(a):
    return None if a is None or (isinstance(a, np.ndarray) and a.size == 0) else a.ctypes.data


class Records:
    """A random interleaved log: transactions with updates then a commit (or an
    abort, or nothing yet), other record kinds mixed in."""

    def __init__(self, seed, n_txn, K, D, crdt, sparse, foreign=0.0):
        """foreign: the fraction of updates whose key is outside [0, K) -- not
        this partition's; the ingest skips them."""
        rng = np.random.default_rng(seed)
        W = (D + 63) // 64
        self.K, self.D, self.W, self.crdt, self.sparse = K, D, W, crdt, sparse
        streams = []
        for t in range(n_txn):
            txid = 1000 + 7 * t
            recs = [("u", txid, int(rng.integers(K, K + 50) if rng.random() < foreign
                                    else rng.integers(0, K)))
                    for _ in range(int(rng.integers(1, 5)))]
            if rng.random() < 0.1:
                recs.append(("o", txid, 0))  # prepare
            end = rng.random()
            if end < 0.8:
                recs.append(("c", txid, 0))
            elif end < 0.9:
                recs.append(("o", txid, 0))  # abort
            streams.append(recs)
        # interleave keeping each transaction's order
        order = []
        pos = [0] * n_txn
        live = list(range(n_txn))
        while live:
            i = live[int(rng.integers(0, len(live)))]
            order.append(streams[i][pos[i]])
            pos[i] += 1
            if pos[i] == len(streams[i]):
                live.remove(i)
        n = len(order)
        self.n = n
        self.kind = np.array([{"u": 1, "c": 2, "o": 0}[r[0]] for r in order], np.uint8)
        self.txid = np.array([r[1] for r in order], np.uint64)
        self.key = np.array([r[2] for r in order], np.uint64)
        self.commit_dc = rng.integers(0, D, n).astype(np.uint32)
        self.ss = (1_000_000 + rng.integers(0, 2000, (n, D))).astype(np.uint64)
        self.commit_time = self.ss.max(axis=1) + rng.integers(1, 50, n).astype(np.uint64)
        self.ss_mask = None
        if sparse:
            self.ss_mask = np.zeros((n, W), np.uint64)
            pres = rng.random((n, D)) >= 0.25
            for d in range(D):
                self.ss_mask[:, d >> 6] |= pres[:, d].astype(np.uint64) << np.uint64(d & 63)
        if crdt == _abi.COUNTER_PN:
            self.eff = rng.integers(-1000, 1000, n).astype(np.int64)
            self.tag = self.add_tok = self.rem_off = self.rem_tok = None
        else:
            self.eff = None
            self.tag = rng.integers(0, 8, n).astype(np.uint32)
            self.add_tok = np.where(rng.random(n) < 0.7, np.arange(n) + 1, 0).astype(np.uint64)
            lens = rng.integers(0, 4, n)
            self.rem_off = np.zeros(n + 1, np.uint32)
            self.rem_off[1:] = np.cumsum(lens)
            self.rem_tok = rng.integers(1, n + 1, max(int(self.rem_off[-1]), 1)).astype(np.uint64)
        self.max_t = self.max_m = None

    def with_max(self, seed):
        rng = np.random.default_rng(seed)
        self.max_t = (1_000_000 + rng.integers(1200, 2200, (self.K, self.D))).astype(np.uint64)
        self.max_t[rng.random(self.K) < 0.5] = 1_002_100  # half the keys admit every commit
        if self.sparse:
            self.max_m = np.zeros((self.K, self.W), np.uint64)
            pres = rng.random((self.K, self.D)) >= 0.05
            for d in range(self.D):
                self.max_m[:, d >> 6] |= pres[:, d].astype(np.uint64) << np.uint64(d & 63)
        return self

    def struct(self, arrs=None):
        a = arrs or self.__dict__
        s = _abi.AgnLogRecords()
        s.n = self.n
        for f in ("kind", "txid", "key", "commit_dc", "commit_time", "ss", "ss_mask", "eff",
                  "tag", "add_tok", "rem_off", "rem_tok"):
            v = a.get(f)
            setattr(s, f, v if isinstance(v, int) else ptr(v))
        return s

    def out_arrays(self):
        n, D, W = self.n, self.D, self.W
        o = {"key_off": np.zeros(self.K + 1, np.uint64), "oc": np.zeros((n, D), np.uint64),
             "oc_mask": np.zeros((n, W), np.uint64) if self.sparse else None,
             "op_id": np.zeros(n, np.uint32), "txid": np.zeros(n, np.uint64)}
        if self.crdt == _abi.COUNTER_PN:
            o["eff"] = np.zeros(n, np.int64)
        else:
            o.update({"tag": np.zeros(n, np.uint32), "add_tok": np.zeros(n, np.uint64),
                      "rem_off": np.zeros(n + 1, np.uint32),
                      "rem_tok": np.zeros(max(int(self.rem_off[-1]), 1), np.uint64)})
        return o


def log_struct_of(arrs):
    s = _abi.AgnLog()
    for f, v in arrs.items():
        setattr(s, f, v if isinstance(v, int) else ptr(v))
    return s


def oracle_ingest(lib, rc, base):
    o = rc.out_arrays()
    s = log_struct_of(o)
    assert lib.oracle_log_ingest(C.byref(rc.struct()), rc.crdt, rc.D, rc.K, ptr(rc.max_t),
                                 ptr(rc.max_m), base, C.byref(s)) == 0
    return o, int(s.n_entries)


def vc(row, mrow, D):
    return {d: int(row[d]) for d in range(D)
            if mrow is None or (int(mrow[d >> 6]) >> (d & 63)) & 1}


def py_filter_terms(rc):
    """filter_terms_for_key + handle_update + handle_commit, literally:
    Ops :: dict(TxId -> [update]), CommittedOpsDict :: dict(Key -> [payload])."""
    ops, committed = {}, {}
    for x in range(rc.n):
        t = int(rc.txid[x])
        if rc.kind[x] == _abi.REC_UPDATE:
            ops.setdefault(t, []).append(x)           # dict:append(TxId, OpPayload, Ops)
        elif rc.kind[x] == _abi.REC_COMMIT:
            if t not in ops:                            # dict:find -> error
                continue
            ss = vc(rc.ss[x], None if rc.ss_mask is None else rc.ss_mask[x], rc.D)
            for u in ops[t]:
                k = int(rc.key[u])
                if k >= rc.K:                               # another partition's key
                    continue
                if rc.max_t is not None:
                    mx = vc(rc.max_t[k], None if rc.max_m is None else rc.max_m[k], rc.D)
                    if not po.vc_le(ss, mx):            # check_max_time
                        continue
                oc = dict(ss)
                oc[int(rc.commit_dc[x])] = int(rc.commit_time[x])  # commit_time = {DcId, T}
                committed.setdefault(k, []).append((u, oc))
            del ops[t]                                   # dict:erase(TxId, Ops)
    return committed


CASES = [(_abi.COUNTER_PN, 3, False, False), (_abi.COUNTER_PN, 8, True, True),
         (_abi.SET_AW, 5, False, True), (_abi.REGISTER_MV, 16, True, False),
         (_abi.COUNTER_PN, 70, True, True)]


@pytest.mark.parametrize("foreign", [0.0, 0.05])
@pytest.mark.parametrize("crdt,D,sparse,use_max", CASES)
def test_oracle_ingest_vs_dict_transcription(oracle_lib, crdt, D, sparse, use_max, foreign):
    rc = Records(D * 5 + crdt, 400, 37, D, crdt, sparse, foreign)
    if use_max:
        rc.with_max(D)
    out, n_out = oracle_ingest(oracle_lib, rc, 0)
    want = py_filter_terms(rc)
    assert n_out == sum(len(v) for v in want.values())
    for k in range(rc.K):
        a, b = int(out["key_off"][k]), int(out["key_off"][k + 1])
        lst = want.get(k, [])
        assert b - a == len(lst), k
        for j, (u, oc) in enumerate(lst):
            e = a + j
            assert int(out["op_id"][e]) == j  # reverse_and_add_op_id numbering (oldest = 0)
            assert int(out["txid"][e]) == int(rc.txid[u])
            got = vc(out["oc"][e], None if out["oc_mask"] is None else out["oc_mask"][e], D)
            assert got == (oc if sparse else {d: oc.get(d, 0) for d in range(D)})
            if crdt == _abi.COUNTER_PN:
                assert int(out["eff"][e]) == int(rc.eff[u])
            else:
                assert int(out["tag"][e]) == int(rc.tag[u])
                r0, r1 = int(out["rem_off"][e]), int(out["rem_off"][e + 1])
                assert list(out["rem_tok"][r0:r1]) == \
                    list(rc.rem_tok[int(rc.rem_off[u]):int(rc.rem_off[u + 1])])
    assert 0 < n_out < int((rc.kind == _abi.REC_UPDATE).sum())


@pytest.mark.gpu
@pytest.mark.parametrize("crdt,D,sparse,use_max", CASES + [(_abi.SET_AW, 16, False, False)])
@pytest.mark.parametrize("base", [0, 1])
def test_ingest_gpu_vs_oracle(eng, oracle_lib, crdt, D, sparse, use_max, base):
    # base 1 also carries updates of keys outside the partition
    rc = Records(D * 11 + crdt + base, 20000, 3000, D, crdt, sparse, 0.03 * base)
    if use_max:
        rc.with_max(D + 1)
    want, n_out = oracle_ingest(oracle_lib, rc, base)
    dev = {f: eng.upload(getattr(rc, f)) for f in ("kind", "txid", "key", "commit_dc",
                                                  "commit_time", "ss", "ss_mask", "eff", "tag",
                                                  "add_tok", "rem_off", "rem_tok")
           if getattr(rc, f) is not None}
    rs = rc.struct({f: b.ptr for f, b in dev.items()})
    outs = {f: (eng.empty(a.nbytes), a.dtype, a.shape) for f, a in want.items() if a is not None}
    os_ = log_struct_of({f: b.ptr for f, (b, _, _) in outs.items()})
    mt = eng.upload(rc.max_t) if rc.max_t is not None else None
    mm = eng.upload(rc.max_m) if rc.max_m is not None else None
    tot = eng.empty(16)
    rcode = eng.lib.agn_log_ingest(eng.ctx, C.byref(rs), crdt, D, rc.K, mt.ptr if mt else None,
                                   mm.ptr if mm else None, base, C.byref(os_), tot.ptr, None)
    assert rcode == 0, eng.lib.agn_last_error()
    eng.sync()
    totals = eng.download(tot, np.uint64, (2,))
    assert int(totals[0]) == n_out
    for f, (b, dt, shape) in outs.items():
        got = eng.download(b, dt, shape)
        w = want[f]
        if f == "key_off":
            assert np.array_equal(got, w)
        elif f == "rem_off":
            assert np.array_equal(got[:n_out + 1], w[:n_out + 1])
        elif f == "rem_tok":
            nr = int(w[0:1].size and want["rem_off"][n_out])
            assert int(totals[1]) == nr
            assert np.array_equal(got[:nr], w[:nr])
        else:
            assert np.array_equal(got[:n_out], w[:n_out]), f
