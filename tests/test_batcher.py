"""SURVEY.md §8(b) threading: many concurrent read servers (READ_CONCURRENCY =
20 per partition, include/antidote.hrl:28) calling materializer_vnode:read/6
per key, coalesced by agn_batcher into batched kernels over the engine-owned
op log, with a concurrent writer appending (update/2).  Every per-key result
must equal the C oracle's for the same ops, and reads must see the writes
that precede them (update/2 is a sync_command before the read)."""
import ctypes as C
import threading
from types import SimpleNamespace

import numpy as np
import pytest

from antidote_amd import _abi
from antidote_amd.encode import alloc_result, log_struct, read_struct, result_struct, state_capacity
from antidote_amd.engine import Batcher, OpLog
from synth import compare, random_case
from test_oplog import append_ops, interleave, ops_of, renumbered

pytestmark = pytest.mark.gpu


def oracle(oracle_lib, log, req, sparse):
    cap = state_capacity(log, req)
    res = alloc_result(req.n_req, log.n_dcs, sparse=sparse, cap_off=cap)
    ls, rs, os_ = log_struct(log), read_struct(req, sparse=sparse), result_struct(res)
    if log.oc_mask is None:
        ls.oc_mask = None
    assert oracle_lib.oracle_materialize(C.byref(ls), C.byref(rs), C.byref(os_), 4) == 0
    return res, cap


def key_read_args(req, i, sparse):
    kw = dict(R=req.R[i], txid=int(req.txid[i]) if req.txid is not None else 0)
    if sparse and req.R_mask is not None:
        kw["R_mask"] = req.R_mask[i]
    if req.sct is not None and not (req.sct_ignore is not None and req.sct_ignore[i]):
        kw["sct"] = req.sct[i]
        if sparse and req.sct_mask is not None:
            kw["sct_mask"] = req.sct_mask[i]
    if req.base_value is not None:
        kw["base_value"] = int(req.base_value[i])
    if req.base_off is not None:
        a, b = int(req.base_off[i]), int(req.base_off[i + 1])
        kw["base_tag"], kw["base_tok"] = req.base_tag[a:b], req.base_tok[a:b]
    return kw


def gather(results, n, D, cap):
    """Per-key batcher results -> a ResultArrays-like object for synth.compare."""
    W = (D + 63) // 64
    total = int(cap[-1]) if cap is not None else 0
    r = SimpleNamespace(value=np.zeros(n, np.int64), hole=np.zeros(n, np.int64),
                        lastct=np.zeros((n, D), np.uint64), lastct_mask=np.zeros((n, W), np.uint64),
                        count=np.zeros(n, np.uint32), flags=np.zeros(n, np.uint32),
                        err_pos=np.zeros(n, np.uint32), out_off=cap,
                        out_n=np.zeros(n, np.uint32), out_tag=np.zeros(max(total, 1), np.uint32),
                        out_tok=np.zeros(max(total, 1), np.uint64))
    for i, g in enumerate(results):
        for f in ("value", "hole", "count", "flags", "err_pos", "out_n"):
            getattr(r, f)[i] = g[f]
        r.lastct[i], r.lastct_mask[i] = g["lastct"], g["lastct_mask"]
        if cap is not None and g["out_n"]:
            o = int(cap[i])
            r.out_tag[o:o + g["out_n"]] = g["out_tag"]
            r.out_tok[o:o + g["out_n"]] = g["out_tok"]
    return r


def run_threads(n_threads, fn, items):
    errs = []

    def body(part):
        try:
            for x in part:
                fn(x)
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    ts = [threading.Thread(target=body, args=(items[t::n_threads],)) for t in range(n_threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise errs[0]


CASES = [(_abi.COUNTER_PN, 8, False), (_abi.COUNTER_PN, 5, True), (_abi.SET_AW, 16, False),
         (_abi.SET_AW, 6, True), (_abi.REGISTER_MV, 8, True)]


@pytest.mark.parametrize("crdt,D,sparse", CASES)
def test_batcher_concurrent_reads_vs_oracle(eng, oracle_lib, crdt, D, sparse):
    rng = np.random.default_rng(3 * D + crdt)
    log, req, _ = random_case(17 * D + crdt, crdt, 300, D, 40, sparse=sparse, warm=0.4, txid=0.2,
                              base=0.3, multi=0.2 if crdt == _abi.SET_AW else 0.0)
    with OpLog(eng, crdt, D, log.n_keys, sparse=sparse, init_slots=8) as ol:
        got = append_ops(ol, log, interleave(rng, ops_of(log)), rng, flush_p=0.3)
        log2 = renumbered(log, got)
        want, cap = oracle(oracle_lib, log2, req, sparse)
        results = [None] * req.n_req
        with Batcher(ol, max_batch=64, max_wait_us=300) as bt:
            def one(i):
                k = int(req.keys[i]) if req.keys is not None else i
                oc = int(cap[i + 1] - cap[i]) if cap is not None else 0
                results[i] = bt.read(k, out_cap=oc, **key_read_args(req, i, sparse))
            run_threads(20, one, list(range(req.n_req)))
            st = bt.stats()
        assert st["reads"] == req.n_req
        assert st["batches"] < req.n_req  # the reads were coalesced
        got_r = gather(results, req.n_req, D, cap)
        # the batcher names the failing op by its id (agn_key_result.err_pos,
        # ABI v5), the oracle by its entry in the log
        bad = want.err_pos != np.uint32(0xFFFFFFFF)
        want.err_pos[bad] = np.asarray(log2.op_id)[want.err_pos[bad]]
        assert not compare(crdt, D, got_r, want, sparse, req.n_req)


def test_batcher_capacity_error(eng):
    log, req, _ = random_case(5, _abi.SET_AW, 4, 4, 30, empty=0.0)
    with OpLog(eng, _abi.SET_AW, 4, log.n_keys) as ol:
        append_ops(ol, log, ops_of(log), np.random.default_rng(0))
        with Batcher(ol, max_batch=8) as bt:
            big = 10 ** 9
            full = bt.read(0, R=np.full(4, big, np.uint64), out_cap=64)
            assert full["out_n"] > 0
            with pytest.raises(Exception, match="out_cap"):
                bt.read(0, R=np.full(4, big, np.uint64), out_cap=0)
            with pytest.raises(Exception):
                bt.read(99, R=np.full(4, big, np.uint64))


def test_batcher_reads_see_preceding_writes(eng):
    """A writer thread appends increments and then reads its own key through
    the batcher while 8 reader threads hammer other keys; every read of the
    writer's key must count every increment appended before it."""
    D, K = 4, 64
    big = np.full(D, 10 ** 12, np.uint64)
    with OpLog(eng, _abi.COUNTER_PN, D, K, init_slots=2) as ol:
        with Batcher(ol, max_batch=32, max_wait_us=100) as bt:
            stop = threading.Event()
            errs = []

            def writer():
                try:
                    for j in range(1, 301):
                        k = j % 4
                        oc = np.full((1, D), 1000 + j, np.uint64)
                        ol.append(np.array([k], np.uint64), oc, eff=np.array([j], np.int64))
                        r = bt.read(k, R=big)
                        want = sum(x for x in range(1, j + 1) if x % 4 == k)
                        assert r["value"] == want and r["count"] == len(
                            [x for x in range(1, j + 1) if x % 4 == k]), (j, r["value"], want)
                except Exception as e:  # noqa: BLE001
                    errs.append(e)
                finally:
                    stop.set()

            def reader(t):
                try:
                    while not stop.is_set():
                        r = bt.read(4 + t, R=big)
                        assert r["count"] == 0 and r["value"] == 0
                except Exception as e:  # noqa: BLE001
                    errs.append(e)
            ts = [threading.Thread(target=writer)] + \
                [threading.Thread(target=reader, args=(t,)) for t in range(8)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
            assert not errs, errs[0]
            assert bt.stats()["reads"] > 300
