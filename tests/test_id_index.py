"""agn_log.key_id0 (ABI v3): the per-key consecutive-op-id index the counter
kernel uses to derive NewLastOp (materialize/4's hole, src/clocksi_materializer.erl:
89-101, 157-197) without a dependent op_id load.  The index kernel is checked
against a numpy restatement, and materialize with the index must equal the C
oracle (and the same read without the index) on logs that mix consecutive ids
(ets:update_counter, src/materializer_vnode.erl:630), GC gaps (:576-585),
empty keys and ids at the top of the u32 range."""
import ctypes as C

import numpy as np
import pytest

from antidote_amd import _abi
from antidote_amd.encode import alloc_result, log_struct, read_struct, result_struct
from synth import compare, random_case


def expected_index(key_off, key_len, op_id):
    K = len(key_len) if key_len is not None else len(key_off) - 1
    out = np.full(K, _abi.ID0_NONE, np.uint32)
    for k in range(K):
        a = int(key_off[k])
        n = int(key_len[k]) if key_len is not None else int(key_off[k + 1]) - a
        if n == 0:
            continue
        id0 = int(op_id[a])
        if id0 + n - 1 >= _abi.ID0_NONE:
            continue
        if np.array_equal(op_id[a:a + n].astype(np.int64), id0 + np.arange(n, dtype=np.int64)):
            out[k] = id0
    return out


def mixed_ids(log, seed, p_consec=0.6, p_top=0.05):
    """Rewrite op ids: a fraction of keys get consecutive ids from a random
    base (some ending exactly at or past 2^32 - 2), the rest keep the gapped
    ids of random_case."""
    rng = np.random.default_rng(seed)
    K = len(log.key_off) - 1
    for k in range(K):
        a, b = int(log.key_off[k]), int(log.key_off[k + 1])
        n = b - a
        if n == 0:
            continue
        u = rng.random()
        if u < p_top:
            top = (1 << 32) - 1 - n + int(rng.integers(0, 2))  # last id = NONE - 1 or NONE
            log.op_id[a:b] = (top + np.arange(n)).astype(np.uint32)
        elif u < p_top + p_consec:
            base = int(rng.integers(1, 1 << 20))
            log.op_id[a:b] = (base + np.arange(n)).astype(np.uint32)
            if n > 2 and rng.random() < 0.2:  # one interior gap (a GC prune)
                j = int(rng.integers(1, n))
                log.op_id[a + j:b] += np.uint32(1)
    return log


def test_expected_index_restatement():
    key_off = np.array([0, 3, 3, 6, 8], np.uint64)
    op_id = np.array([5, 6, 7, 1, 3, 4, 0xFFFFFFFE, 0xFFFFFFFF], np.uint32)
    got = expected_index(key_off, None, op_id)
    assert got.tolist() == [5, _abi.ID0_NONE, _abi.ID0_NONE, _abi.ID0_NONE]
    key_len = np.array([2, 0, 1, 1], np.uint64)
    got = expected_index(key_off, key_len, op_id)
    assert got.tolist() == [5, _abi.ID0_NONE, 1, 0xFFFFFFFE]


@pytest.mark.gpu
@pytest.mark.parametrize("seed,K,nmax", [(1, 500, 150), (2, 64, 1500), (3, 2000, 3)])
def test_index_kernel_vs_numpy(eng, seed, K, nmax):
    log, req, _ = random_case(seed, _abi.COUNTER_PN, K, 4, nmax)
    log = mixed_ids(log, seed)
    d = eng.upload_log(log)
    b = eng.index_ids(d)
    eng.sync()
    got = eng.download(b, np.uint32, (K,))
    want = expected_index(log.key_off, None, log.op_id)
    assert np.array_equal(got, want)
    assert (want != _abi.ID0_NONE).any() and (want == _abi.ID0_NONE).any()


@pytest.mark.gpu
def test_index_kernel_segmented(eng):
    """key_len (segments with slack, the op log's layout)."""
    from antidote_amd.engine import DeviceArrays
    rng = np.random.default_rng(11)
    K, cap = 300, 80
    key_off = (np.arange(K + 1) * cap).astype(np.uint64)
    key_len = rng.integers(0, cap + 1, K).astype(np.uint64)
    op_id = rng.integers(1, 1000, K * cap).astype(np.uint32)
    for k in range(0, K, 2):
        op_id[k * cap:(k + 1) * cap] = (7 + k + np.arange(cap)).astype(np.uint32)
    s = _abi.AgnLog(crdt_type=_abi.COUNTER_PN, n_dcs=1, n_keys=K, n_entries=K * cap)
    bufs = {n: eng.upload(a) for n, a in (("key_off", key_off), ("key_len", key_len),
                                          ("op_id", op_id))}
    for n, bb in bufs.items():
        setattr(s, n, bb.ptr)
    b = eng.index_ids(DeviceArrays(s, bufs))
    eng.sync()
    got = eng.download(b, np.uint32, (K,))
    assert np.array_equal(got, expected_index(key_off, key_len, op_id))


IMPLS = ("auto", "glds", "general")


@pytest.mark.gpu
@pytest.mark.parametrize("impl", IMPLS)
@pytest.mark.parametrize("D", [3, 8])
def test_materialize_with_index_vs_oracle(eng, oracle_lib, monkeypatch, impl, D):
    monkeypatch.delenv("AGN_COUNTER_IMPL", raising=False)
    monkeypatch.setenv("AGN_COUNTER_GLDS", "0")  # "auto": VGPR rows, whatever agn_tune chose
    monkeypatch.delenv("AGN_COUNTER_ID0", raising=False)
    if impl == "general":
        monkeypatch.setenv("AGN_COUNTER_IMPL", "general")
    elif impl == "glds":
        monkeypatch.setenv("AGN_COUNTER_GLDS", "1")
    log, req, _ = random_case(100 + D, _abi.COUNTER_PN, 600, D, 200, warm=0.4, txid=0.3,
                              invalid=0.02, corrupt=0.03, base=0.4, identity=(D == 8))
    log = mixed_ids(log, D)
    dl = eng.upload_log(log)
    dr = eng.upload_read(req, sparse=False)
    dl.struct.oc_mask = None
    res_plain = eng.alloc_result(req.n_req, D, sparse=False)
    eng.materialize(dl, dr, res_plain)
    eng.index_ids(dl)
    res_idx = eng.alloc_result(req.n_req, D, sparse=False)
    eng.materialize(dl, dr, res_idx)
    eng.sync()
    g_plain, g_idx = eng.fetch_result(res_plain), eng.fetch_result(res_idx)

    res_o = alloc_result(req.n_req, D, sparse=False)
    ls, rs, os_ = log_struct(log), read_struct(req, sparse=False), result_struct(res_o)
    ls.oc_mask = None
    assert oracle_lib.oracle_materialize(C.byref(ls), C.byref(rs), C.byref(os_), 4) == 0
    assert not compare(_abi.COUNTER_PN, D, g_idx, res_o, False, req.n_req)
    assert not compare(_abi.COUNTER_PN, D, g_plain, res_o, False, req.n_req)


@pytest.mark.gpu
def test_host_staged_index(eng, oracle_lib):
    """agn_materialize_host stages a host key_id0 like every other log array."""
    log, req, _ = random_case(77, _abi.COUNTER_PN, 400, 5, 120, warm=0.3, base=0.3)
    log = mixed_ids(log, 77)
    idx = expected_index(log.key_off, None, log.op_id)
    res = alloc_result(req.n_req, 5, sparse=False)
    ls, rs, os_ = log_struct(log), read_struct(req, sparse=False), result_struct(res)
    ls.oc_mask = None
    ls.key_id0 = idx.ctypes.data
    assert eng.lib.agn_materialize_host(eng.ctx, C.byref(ls), C.byref(rs), C.byref(os_)) == 0
    res_o = alloc_result(req.n_req, 5, sparse=False)
    ls2, rs2, os2 = log_struct(log), read_struct(req, sparse=False), result_struct(res_o)
    ls2.oc_mask = None
    assert oracle_lib.oracle_materialize(C.byref(ls2), C.byref(rs2), C.byref(os2), 4) == 0
    assert not compare(_abi.COUNTER_PN, 5, res, res_o, False, req.n_req)
