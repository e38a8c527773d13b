"""Host-path concurrency (SURVEY.md §8(b) Threading): the per-key NIF entry
agn_materialize_host called from many threads at once, and the read batcher
sizing set/register outputs while a writer appends to the same keys."""
import ctypes as C
import threading

import numpy as np
import pytest

from antidote_amd import _abi
from antidote_amd.encode import alloc_result, log_struct, read_struct, result_struct
from antidote_amd.engine import Batcher, OpLog
from synth import compare, random_case

pytestmark = pytest.mark.gpu


def test_materialize_host_many_threads(eng, oracle_lib):
    """16 threads x 6 calls of agn_materialize_host (each call borrows a
    stager: its own stream and buffers) on different logs; every result is
    bit-exact against the oracle."""
    cases = []
    for i in range(24):
        crdt = (_abi.COUNTER_PN, _abi.SET_AW, _abi.REGISTER_MV)[i % 3]
        D = (3, 8, 16, 64)[i % 4]
        sparse = i % 5 == 0
        log, req, cap = random_case(900 + i, crdt, 80, D, 50, sparse=sparse, warm=0.3, txid=0.2,
                                    base=0.3, multi=0.15 if crdt == _abi.SET_AW else 0.0)
        want = alloc_result(req.n_req, D, sparse=sparse, cap_off=cap)
        ls, rs, os_ = log_struct(log), read_struct(req, sparse=sparse), result_struct(want)
        if not sparse:
            ls.oc_mask = None
        assert oracle_lib.oracle_materialize(C.byref(ls), C.byref(rs), C.byref(os_), 1) == 0
        cases.append((crdt, D, sparse, log, req, cap, want))
    errs = []

    def body(t):
        try:
            for r in range(6):
                crdt, D, sparse, log, req, cap, want = cases[(t * 7 + r) % len(cases)]
                got = eng.materialize_host(log, req, sparse=sparse, cap_off=cap)
                bad = compare(crdt, D, got, want, sparse, req.n_req)
                assert not bad, (t, r, bad[:3])
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    ts = [threading.Thread(target=body, args=(t,)) for t in range(16)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs[0]


@pytest.mark.parametrize("crdt", [_abi.SET_AW, _abi.REGISTER_MV])
def test_batcher_sizes_outputs_under_concurrent_appends(eng, crdt):
    """A writer appends adds / assigns to the very keys 8 reader threads read.
    The batcher sizes each read's output capacity from the key's length; the
    length must be the one the kernel sees (taken under the flush's lock), so
    no read may come back with AGN_F_ERR_CAPACITY, and a read's live pairs
    never exceed the entries appended before it returned."""
    D, K, N = 4, 6, 600
    big = np.full(D, 10 ** 12, np.uint64)
    appended = [0] * K
    lock = threading.Lock()
    with OpLog(eng, crdt, D, K, init_slots=4) as ol:
        with Batcher(ol, max_batch=16, max_wait_us=50) as bt:
            stop = threading.Event()
            errs = []

            def writer():
                try:
                    for j in range(N):
                        k = j % K
                        oc = np.full((1, D), 1000 + j, np.uint64)
                        with lock:   # counted before it can be read
                            appended[k] += 1
                        # set_aw: a fresh token for a new element (never removed);
                        # register_mv: a concurrent assign (overrides nothing)
                        ol.append(np.array([k], np.uint64), oc, tag=np.array([j], np.uint32),
                                  add_tok=np.array([j + 1], np.uint64),
                                  rem_off=np.array([0, 0], np.uint32), rem_tok=None)
                except Exception as e:  # noqa: BLE001
                    errs.append(e)
                finally:
                    stop.set()

            def reader(t):
                try:
                    while not stop.is_set():
                        k = t % K
                        r = bt.read(k, R=big, out_cap=N)
                        with lock:
                            n_app = appended[k]
                        assert not (r["flags"] & _abi.F_ERR_CAPACITY), r["flags"]
                        assert r["out_n"] == r["count"] <= n_app, (r["out_n"], r["count"], n_app)
                except Exception as e:  # noqa: BLE001
                    errs.append(e)
            ts = [threading.Thread(target=writer)] + \
                [threading.Thread(target=reader, args=(t,)) for t in range(8)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
            assert not errs, errs[0]
            final = [bt.read(k, R=big, out_cap=N)["out_n"] for k in range(K)]
            assert final == appended


def test_batched_reads_concurrent_with_prune_sparse_log(eng):
    """Lock order: a batcher worker reading a sparse log
    counts the batch's mixed-DC-set keys (AGN_HINT_MIXED) under the writer
    lock before it takes the arena shared, so a concurrent agn_oplog_prune
    (writer lock, then the arena exclusively) cannot deadlock with it.  8
    reader threads and one pruning / appending thread on one sparse
    counter_pn log; every thread must finish, and every read's value is the
    sum of the effects appended before it (nothing is ever pruned: the
    thresholds are all 0)."""
    D, K = 4, 8
    W = 1
    big = np.full(D, 10 ** 12, np.uint64)
    with OpLog(eng, _abi.COUNTER_PN, D, K, sparse=True, init_slots=4) as ol:
        # half the keys hold entries of two DC sets (umask 0: "mixed")
        for j in range(64):
            k = j % K
            m = 0b1111 if (k % 2 == 0 or j % 3) else 0b0111
            ol.append(np.array([k], np.uint64), np.full((1, D), 100 + j, np.uint64),
                      oc_mask=np.array([[m]], np.uint64), eff=np.array([1], np.int64))
        prune = eng.upload(np.ones(K, np.uint8))
        thr = eng.upload(np.zeros((K, D), np.uint64))
        tmask = eng.upload(np.full((K, W), ~np.uint64(0), np.uint64))
        with Batcher(ol, max_batch=8, max_wait_us=50) as bt:
            stop = threading.Event()
            errs = []
            n_app = [8] * K

            def gc():
                try:
                    for j in range(300):
                        ol.prune(prune.ptr, thr.ptr, tmask.ptr)
                        k = j % K
                        ol.append(np.array([k], np.uint64), np.full((1, D), 1000 + j, np.uint64),
                                  oc_mask=np.array([[0b1011 if j % 2 else 0b1111]], np.uint64),
                                  eff=np.array([1], np.int64))
                        n_app[k] += 1
                except Exception as e:  # noqa: BLE001
                    errs.append(e)
                finally:
                    stop.set()

            def reader(t):
                try:
                    while not stop.is_set():
                        k = t % K
                        lo = n_app[k]
                        r = bt.read(k, R=big, R_mask=np.array([0b1111], np.uint64))
                        # an append may land before its count does
                        assert lo <= r["value"] <= n_app[k] + 1, (k, lo, r["value"])
                except Exception as e:  # noqa: BLE001
                    errs.append(e)
            ts = [threading.Thread(target=gc, daemon=True)] + \
                [threading.Thread(target=reader, args=(t,), daemon=True) for t in range(8)]
            for t in ts:
                t.start()
            for t in ts:
                t.join(timeout=90)
            assert not any(t.is_alive() for t in ts), "deadlock: reader / prune threads stuck"
            assert not errs, errs[0]
            assert [bt.read(k, R=big, R_mask=np.array([0b1111], np.uint64))["value"]
                    for k in range(K)] == n_app
