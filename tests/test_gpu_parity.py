"""Parity of the HIP engine with the C oracle (and, through it, with the
reference's known answers).  Bit-exact on every output: value / state pairs,
NewLastOp, LastOpCt (+ presence), Count, IsNewSS, error kind and position."""
import ctypes as C

import numpy as np
import pytest

from antidote_amd import _abi
from antidote_amd.encode import alloc_result, log_struct, read_struct, result_struct
from antidote_amd.engine import Engine, free_gen_host, gen_host, host_view
from kat_util import TYPES, OneKeyRun, kats, oracle_fn, py_ops, to_vc
from synth import compare, random_case

pytestmark = pytest.mark.gpu


def gpu_fn(eng):
    def fn(ls, rs, os_):
        return eng.lib.agn_materialize_host(eng.ctx, C.byref(ls), C.byref(rs), C.byref(os_))
    return fn


# ------------------------------------------------------------------ KATs on the GPU
MAT = kats({"materialize", "materialize_chain"})


@pytest.mark.parametrize("c", MAT, ids=[c["name"] for c in MAT])
def test_kat_materialize_gpu(eng, oracle_lib, c):
    from test_oracle_kats import c_materialize_case, check_expect
    r = c_materialize_case(gpu_fn(eng), c)
    check_expect(r, c["expect"])
    assert r == c_materialize_case(oracle_fn(oracle_lib), c)


SYS = kats({"system_seq"})


@pytest.mark.parametrize("c", SYS, ids=[c["name"] for c in SYS])
def test_kat_system_seq_gpu(eng, c):
    from kat_util import system_seq_log
    from oracle import py_oracle as po
    typ = TYPES[c["type"]]
    ops, reads, _ = system_seq_log(c)
    for i in range(len(reads)):
        run = OneKeyRun(c["type"], ops, 1)
        run.add_read(reads[i])
        _, res = run.run(gpu_fn(eng))
        g = run.decode(res, 0)
        want = po.materialize(typ, po.IGNORE, reads[i], po.SnapshotGetResponse(
            ops, len(ops), po.MaterializedSnapshot(0, po.crdt_new(typ)), po.IGNORE, True))
        assert g == want
        exp = c["expect_after"]
        want_v = exp[i] if isinstance(exp, list) else exp.get(str(i + 1))
        if want_v is not None:
            assert po.crdt_value(typ, g[1]) == want_v


TXN = kats({"system_txn"})


@pytest.mark.parametrize("c", TXN, ids=[c["name"] for c in TXN])
def test_kat_system_txn_gpu(eng, oracle_lib, c):
    """Multi-DC / multi-key / multi-update transaction KATs (inter_dc_repl,
    multiple_dcs and pb_client suites) through the HIP path: the asserted
    value and the full materialize/4 tuple of the dict restatement."""
    from test_oracle_kats import system_txn_check
    system_txn_check(c, gpu_fn(eng))


# ------------------------------------------------------------------ randomised differential
# counter_pn runs through every counter kernel: the dense fast path (auto),
# its opt-in LDS-DMA row path (glds, even D only) and the general kernel
COUNTER_IMPLS = ("auto", "glds", "quad", "quad2", "general")
DIFF = []
for crdt in (_abi.COUNTER_PN, _abi.SET_AW, _abi.REGISTER_MV):
    for D in (1, 2, 3, 5, 8, 12, 16, 17, 33, 64, 100, 256):
        for sparse in (False, True):
            impls = COUNTER_IMPLS if crdt == _abi.COUNTER_PN else ("auto",)
            for impl in impls:
                DIFF.append((crdt, D, sparse, impl))


def _set_impl(monkeypatch, impl):
    monkeypatch.delenv("AGN_COUNTER_IMPL", raising=False)
    monkeypatch.delenv("AGN_COUNTER_GLDS", raising=False)
    # "auto" = the VGPR-row dense kernel whatever agn_tune selected in this
    # process; "glds" / "quad" / "quad2" = the LDS-DMA / quad-row / two-
    # requests-per-wave quad-row variants where the shape has them (even D /
    # D = 8), else VGPR rows
    monkeypatch.setenv("AGN_COUNTER_VARIANT",
                       {"glds": "1", "quad": "2", "quad2": "3"}.get(impl, "0"))
    if impl == "general":
        monkeypatch.setenv("AGN_COUNTER_IMPL", "general")


@pytest.fixture(params=COUNTER_IMPLS)
def counter_impl(request, monkeypatch):
    """Run counter cases through each counter kernel (see COUNTER_IMPLS)."""
    _set_impl(monkeypatch, request.param)
    return request.param


@pytest.mark.parametrize("crdt,D,sparse,impl", DIFF)
def test_random_vs_oracle(eng, oracle_lib, monkeypatch, crdt, D, sparse, impl):
    _set_impl(monkeypatch, impl)
    K = 300 if D <= 64 else 120
    nmax = 150 if D <= 16 else 70
    log, req, cap = random_case(7919 * crdt + 31 * D + sparse, crdt, K, D, nmax, sparse=sparse,
                                warm=0.4, txid=0.3, invalid=0.02, corrupt=0.03,
                                multi=0.15 if crdt == _abi.SET_AW else 0.0, base=0.4,
                                identity=(D % 2 == 0))
    res_g = eng.materialize_host(log, req, sparse=sparse, cap_off=cap)
    res_o = alloc_result(req.n_req, D, sparse=sparse, cap_off=cap)
    ls, rs, os_ = log_struct(log), read_struct(req, sparse=sparse), result_struct(res_o)
    if not sparse:
        ls.oc_mask = None
    assert oracle_lib.oracle_materialize(C.byref(ls), C.byref(rs), C.byref(os_), 4) == 0
    bad = compare(crdt, D, res_g, res_o, sparse, req.n_req)
    assert not bad, bad[:10]


@pytest.mark.parametrize("dpl8", [False, True])
@pytest.mark.parametrize("crdt", [_abi.SET_AW, _abi.REGISTER_MV])
@pytest.mark.parametrize("D", [12, 16, 40, 64, 128])
def test_tags_dense_shapes_vs_oracle(eng, oracle_lib, monkeypatch, dpl8, crdt, D):
    """Dense D > 8 tag kernel shapes: 4 DCs per lane (default) and the
    8-per-lane shape (AGN_TAGS_DPL8=1)."""
    if dpl8:
        monkeypatch.setenv("AGN_TAGS_DPL8", "1")
    else:
        monkeypatch.delenv("AGN_TAGS_DPL8", raising=False)
    log, req, cap = random_case(4409 * crdt + D, crdt, 150 if D < 100 else 60, D, 150, warm=0.4,
                                txid=0.3,
                                invalid=0.02, corrupt=0.03, base=0.4,
                                multi=0.15 if crdt == _abi.SET_AW else 0.0)
    _, _, bad = _oracle_vs_gpu(eng, oracle_lib, crdt, D, log, req)
    assert not bad, bad[:10]


def test_long_keys_vs_oracle(eng, oracle_lib, counter_impl):
    """Keys far longer than a wave (1000+ ops, like large_list_test) and
    set_aw state that forces table compaction."""
    for crdt in (_abi.COUNTER_PN, _abi.SET_AW, _abi.REGISTER_MV):
        log, req, cap = random_case(99 + crdt, crdt, 24, 8, 1500, warm=0.3, base=0.3,
                                    n_elems=40, empty=0.0)
        res_g = eng.materialize_host(log, req, sparse=False, cap_off=cap)
        res_o = alloc_result(req.n_req, 8, sparse=False, cap_off=cap)
        ls, rs, os_ = log_struct(log), read_struct(req, sparse=False), result_struct(res_o)
        ls.oc_mask = None
        oracle_lib.oracle_materialize(C.byref(ls), C.byref(rs), C.byref(os_), 4)
        assert not compare(crdt, 8, res_g, res_o, False, req.n_req)


@pytest.mark.parametrize("variant", [None, "2", "3"])
@pytest.mark.parametrize("K", [1, 2, 301])
def test_quad_pairs_vs_oracle(eng, oracle_lib, monkeypatch, variant, K):
    """D = 8 quad rows with a request keys array and odd / tiny batches: the
    two-requests-per-wave kernel's last wave has one request; cold and warm
    requests mixed (variant None = the default choice: quad2 for a warm batch)."""
    monkeypatch.delenv("AGN_COUNTER_IMPL", raising=False)
    monkeypatch.delenv("AGN_COUNTER_GLDS", raising=False)
    if variant is None:
        monkeypatch.delenv("AGN_COUNTER_VARIANT", raising=False)
    else:
        monkeypatch.setenv("AGN_COUNTER_VARIANT", variant)
    log, req, cap = random_case(6151 + K, _abi.COUNTER_PN, K, 8, 200, warm=0.5, txid=0.3,
                                invalid=0.02, corrupt=0.05, base=0.4, identity=False)
    _, _, bad = _oracle_vs_gpu(eng, oracle_lib, _abi.COUNTER_PN, 8, log, req)
    assert not bad, bad[:10]


def _oracle_vs_gpu(eng, oracle_lib, crdt, D, log, req, sparse=False):
    from antidote_amd.encode import state_capacity
    cap = state_capacity(log, req)
    res_g = eng.materialize_host(log, req, sparse=sparse, cap_off=cap)
    res_o = alloc_result(req.n_req, D, sparse=sparse, cap_off=cap)
    ls, rs, os_ = log_struct(log), read_struct(req, sparse=sparse), result_struct(res_o)
    if not sparse:
        ls.oc_mask = None
    assert oracle_lib.oracle_materialize(C.byref(ls), C.byref(rs), C.byref(os_), 4) == 0
    return res_g, res_o, compare(crdt, D, res_g, res_o, sparse, req.n_req)


@pytest.mark.parametrize("crdt,D,sparse", [(_abi.COUNTER_PN, 8, False), (_abi.COUNTER_PN, 4, False),
                                            (_abi.COUNTER_PN, 3, False), (_abi.COUNTER_PN, 8, True),
                                            (_abi.SET_AW, 16, False)])
def test_tune_vs_oracle(eng, oracle_lib, monkeypatch, crdt, D, sparse):
    """agn_tune times the path's kernel variants on the batch, leaves the
    batch's results in `out` (bit-exact vs the oracle) and its selection then
    drives agn_materialize (results unchanged)."""
    monkeypatch.delenv("AGN_COUNTER_GLDS", raising=False)
    monkeypatch.delenv("AGN_COUNTER_VARIANT", raising=False)
    monkeypatch.delenv("AGN_COUNTER_IMPL", raising=False)
    log, req, cap = random_case(4243 + 7 * D + crdt, crdt, 400, D, 150, sparse=sparse, warm=0.4,
                                txid=0.3, invalid=0.02, corrupt=0.03, base=0.4,
                                identity=(D % 2 == 0))
    res_o = alloc_result(req.n_req, D, sparse=sparse, cap_off=cap)
    ls, rs, os_ = log_struct(log), read_struct(req, sparse=sparse), result_struct(res_o)
    if not sparse:
        ls.oc_mask = None
    assert oracle_lib.oracle_materialize(C.byref(ls), C.byref(rs), C.byref(os_), 4) == 0
    dl, dr = eng.upload_log(log), eng.upload_read(req, sparse=sparse)
    res = eng.alloc_result(req.n_req, D, sparse=sparse, cap_off=cap)
    choice, ms = eng.tune(dl, dr, res, rounds=2)
    tunable = crdt == _abi.COUNTER_PN and D % 2 == 0 and not sparse
    assert choice in ((0, 1, 2) if tunable else (-1,))
    if tunable:
        assert ms[0] > 0 and ms[1] > 0 and (ms[2] > 0) == (D == 8)
    bad = compare(crdt, D, eng.fetch_result(res), res_o, sparse, req.n_req)
    assert not bad, bad[:10]
    res2 = eng.alloc_result(req.n_req, D, sparse=sparse, cap_off=cap)
    eng.materialize(dl, dr, res2)
    eng.sync()
    bad = compare(crdt, D, eng.fetch_result(res2), res_o, sparse, req.n_req)
    assert not bad, bad[:10]


@pytest.mark.parametrize("crdt", [_abi.SET_AW, _abi.REGISTER_MV])
@pytest.mark.parametrize("D", [8, 16, 64])
def test_large_live_state_slow_path(eng, oracle_lib, crdt, D):
    """Live state beyond the fast table (CAP - 64 = 192 pairs): the key is
    handed to the 4096-slot pass through the device worklist."""
    log, req, _ = random_case(4242 + crdt + D, crdt, 12, D, 1500, base=0.5, n_elems=600,
                              empty=0.0, warm=0.3)
    log.rem_off[:] = 0  # no removals: every included add stays live
    log.rem_tok = np.zeros(1, np.uint64)
    res_g, res_o, bad = _oracle_vs_gpu(eng, oracle_lib, crdt, D, log, req)
    assert not bad, bad[:5]
    assert int(res_o.out_n.max()) > 256  # the slow path really ran


@pytest.mark.parametrize("crdt", [_abi.SET_AW, _abi.REGISTER_MV])
@pytest.mark.parametrize("sparse", [False, True])
def test_repeated_tokens(eng, oracle_lib, crdt, sparse):
    """A token added twice stays twice in the sequential fold (set_aw appends,
    register_mv insert_sorted); a removal kills every earlier copy only."""
    D = 5
    log, req, _ = random_case(77 + crdt + 2 * sparse, crdt, 200, D, 120, base=0.3, sparse=sparse,
                              warm=0.3, n_elems=4)
    rng = np.random.default_rng(9)
    for k in range(len(log.key_off) - 1):
        a, b = int(log.key_off[k]), int(log.key_off[k + 1])
        adds = [e for e in range(a, b) if log.add_tok[e] != 0]
        for j, e in enumerate(adds[1:], 1):
            if rng.random() < 0.3:
                log.add_tok[e] = log.add_tok[adds[int(rng.integers(0, j))]]
    _, _, bad = _oracle_vs_gpu(eng, oracle_lib, crdt, D, log, req, sparse=sparse)
    assert not bad, bad[:5]


def test_empty_batch_and_empty_log(eng):
    log, req, cap = random_case(5, _abi.COUNTER_PN, 10, 4, 0, empty=1.0)
    res = eng.materialize_host(log, req, sparse=False)
    assert (res.count == 0).all() and (res.hole == 0).all()
    assert ((res.flags & _abi.F_CT_IGNORE) > 0).sum() == int((req.sct_ignore == 1).sum())


# ------------------------------------------------------------------ generator
def _arrays(log, req, cfg, dev, eng):
    D, K, N = cfg.n_dcs, cfg.n_keys, cfg.ops_per_key
    E = K * N
    if dev:
        g = lambda p, dt, n: eng.download(type("B", (), {"ptr": p})(), dt, (n,))  # noqa: E731
    else:
        g = lambda p, dt, n: host_view(p, dt, n).copy()  # noqa: E731
    out = {"key_off": g(log.key_off, np.uint64, K + 1), "oc": g(log.oc, np.uint64, E * D),
           "op_id": g(log.op_id, np.uint32, E), "R": g(req.R, np.uint64, K * D)}
    if cfg.crdt_type == _abi.COUNTER_PN:
        out["eff"] = g(log.eff, np.int64, E)
    else:
        out["tag"] = g(log.tag, np.uint32, E)
        out["add_tok"] = g(log.add_tok, np.uint64, E)
        ro = g(log.rem_off, np.uint32, E + 1)
        out["rem_off"] = ro
        out["rem_tok"] = g(log.rem_tok, np.uint64, int(ro[-1]))
    if cfg.warm:
        out["sct"] = g(req.sct, np.uint64, K * D)
    return out


@pytest.mark.parametrize("crdt,D,N,warm", [(1, 8, 64, 0), (1, 3, 100, 1), (2, 16, 256, 0),
                                           (3, 64, 100, 1)])
def test_device_generator_matches_host(eng, crdt, D, N, warm):
    cfg = _abi.AgnGenCfg(crdt_type=crdt, n_dcs=D, n_keys=777, ops_per_key=N, n_elems=32 if
                         crdt == 2 else 16, seed=20250112 + crdt, key_base=5, key_stride=3,
                         warm=warm)
    dl, dr = eng.gen_dev(cfg)
    hl, hr = gen_host(cfg)
    try:
        a = _arrays(dl, dr, cfg, True, eng)
        b = _arrays(hl, hr, cfg, False, eng)
        for k in a:
            assert np.array_equal(a[k], b[k]), k
    finally:
        eng.free_gen(dl, dr)
        free_gen_host(hl, hr)


# ------------------------------------------------------------------ full-size configs
def _run_dev(eng, cfg):
    """Generate on device, materialize on device, return (log, req, device result)."""
    dl, dr = eng.gen_dev(cfg)
    K, D = cfg.n_keys, cfg.n_dcs
    cap = None
    if cfg.crdt_type != _abi.COUNTER_PN:
        # capacity = adds per key + 0 base: bound by ops_per_key
        cap = np.arange(K + 1, dtype=np.uint64) * np.uint64(cfg.ops_per_key)
    res = eng.alloc_result(K, D, sparse=False, cap_off=cap)
    eng.materialize(dl, dr, res)
    eng.sync()
    return dl, dr, res


def _sampled_oracle(oracle_lib, cfg, keys, cap_per_key):
    """Host-generate only the sampled keys (same SplitMix64 streams) and run
    the oracle on them."""
    outs = []
    for k in keys:
        c1 = _abi.AgnGenCfg(crdt_type=cfg.crdt_type, n_dcs=cfg.n_dcs, n_keys=1,
                            ops_per_key=cfg.ops_per_key, n_elems=cfg.n_elems, seed=cfg.seed,
                            key_base=cfg.key_base + int(k) * cfg.key_stride,
                            key_stride=cfg.key_stride, warm=cfg.warm)
        hl, hr = gen_host(c1)
        capo = np.array([0, cap_per_key], np.uint64) if cap_per_key else None
        r = alloc_result(1, cfg.n_dcs, sparse=False, cap_off=capo)
        os_ = result_struct(r)
        assert oracle_lib.oracle_materialize(C.byref(hl), C.byref(hr), C.byref(os_), 1) == 0
        free_gen_host(hl, hr)
        outs.append(r)
    return outs


FULL = [
    # BASELINE cfg2: counter_pn 10M keys x 64 ops, D=8
    dict(crdt_type=1, n_dcs=8, n_keys=10_000_000, ops_per_key=64, n_elems=0, seed=20250113),
    # the same warm (SCT = max oc of a random earlier prefix): two requests per wave
    dict(crdt_type=1, n_dcs=8, n_keys=10_000_000, ops_per_key=64, n_elems=0, seed=20250113,
         warm=1),
    # BASELINE cfg3: set_aw 1M keys x 256 ops, D=16, 32 elems
    dict(crdt_type=2, n_dcs=16, n_keys=1_000_000, ops_per_key=256, n_elems=32, seed=20250114),
    # BASELINE cfg4 (one GPU's shard at G=8): register_mv 125k keys x 100 ops, D=64
    dict(crdt_type=3, n_dcs=64, n_keys=125_000, ops_per_key=100, n_elems=16, seed=20250115,
         key_stride=8),
    # cfg3 / cfg4 warm (SCT rows: the tags kernels' warm filter at full size)
    dict(crdt_type=2, n_dcs=16, n_keys=1_000_000, ops_per_key=256, n_elems=32, seed=20250114,
         warm=1),
    dict(crdt_type=3, n_dcs=64, n_keys=125_000, ops_per_key=100, n_elems=16, seed=20250115,
         key_stride=8, warm=1),
]


@pytest.mark.parametrize("spec", FULL, ids=["cfg2_counter", "cfg2_counter_warm", "cfg3_set_aw", "cfg4_register_mv",
                              "cfg3_set_aw_warm", "cfg4_register_mv_warm"])
def test_full_size_sampled_parity(eng, oracle_lib, spec):
    cfg = _abi.AgnGenCfg(**{"key_base": 0, "key_stride": 1, "warm": 0, **spec})
    dl, dr, res = _run_dev(eng, cfg)
    try:
        K, D = cfg.n_keys, cfg.n_dcs
        flags = eng.download(res.bufs["flags"], np.uint32, (K,))
        count = eng.download(res.bufs["count"], np.uint32, (K,))
        # size-independent properties over every key
        assert not (flags & (_abi.F_ERR_UNEXPECTED | _abi.F_ERR_CORRUPTED |
                             _abi.F_ERR_CAPACITY)).any()
        assert (count <= cfg.ops_per_key).all()
        assert (((flags & _abi.F_NEWSS) > 0) == (count > 0)).all()
        inc = count.mean() / cfg.ops_per_key
        # "random snapshot VCs": neither all nor none (warm: only the ops past SCT)
        assert (0.01 if cfg.warm else 0.2) < inc < 0.8, inc
        # bit-exact on a random sample of keys
        rng = np.random.default_rng(cfg.seed)
        sample = np.sort(rng.choice(K, 64, replace=False))
        sample[0], sample[-1] = 0, K - 1
        cap = cfg.ops_per_key if cfg.crdt_type != 1 else 0
        want = _sampled_oracle(oracle_lib, cfg, sample, cap)
        full = eng.fetch_result(res)
        for j, k in enumerate(sample):
            w = want[j]
            assert int(full.flags[k]) == int(w.flags[0])
            assert int(full.hole[k]) == int(w.hole[0])
            assert int(full.count[k]) == int(w.count[0])
            assert np.array_equal(full.lastct[k], w.lastct[0])
            if cfg.crdt_type == 1:
                assert int(full.value[k]) == int(w.value[0])
            else:
                n = int(full.out_n[k])
                o = int(full.out_off[k])
                assert n == int(w.out_n[0])
                assert np.array_equal(full.out_tag[o:o + n], w.out_tag[:n])
                assert np.array_equal(full.out_tok[o:o + n], w.out_tok[:n])
    finally:
        eng.free_gen(dl, dr)
        for b in res.bufs.values():
            b.free()


CFG1 = dict(crdt_type=1, n_dcs=3, n_keys=10_000, ops_per_key=100, n_elems=0, seed=20250112)


@pytest.mark.parametrize("warm", [0, 1], ids=["cold", "warm"])
def test_cfg1_all_keys_parity(eng, oracle_lib, warm):
    """BASELINE cfg1 (the reference's CPU-runnable case: counter_pn, 10k keys x
    100 ops, 3-DC clocks): every key generated on the device and materialized
    by the HIP path, bit-exact against the oracle on the host-generated log."""
    cfg = _abi.AgnGenCfg(**{"key_base": 0, "key_stride": 1, **CFG1, "warm": warm})
    dl, dr, res = _run_dev(eng, cfg)
    try:
        got = eng.fetch_result(res)
        hl, hr = gen_host(cfg)
        want = alloc_result(cfg.n_keys, cfg.n_dcs, sparse=False)
        assert oracle_lib.oracle_materialize(C.byref(hl), C.byref(hr),
                                             C.byref(result_struct(want)), 4) == 0
        free_gen_host(hl, hr)
        bad = compare(1, cfg.n_dcs, got, want, False, cfg.n_keys)
        assert not bad, bad[:10]
        inc = want.count.mean() / cfg.ops_per_key
        assert 0.2 < inc < 0.8, inc
    finally:
        eng.free_gen(dl, dr)
        for b in res.bufs.values():
            b.free()


# ------------------------------------------------------------------ block orders
BULK = [
    # counter_pn just past the 2^20-request threshold (runs of 64 blocks per
    # XCD), a ragged grid: a tail past the last whole super-run of 8 runs
    dict(crdt_type=1, n_dcs=8, n_keys=(1 << 20) + 12_345, ops_per_key=8, n_elems=0, seed=777),
    dict(crdt_type=1, n_dcs=8, n_keys=(1 << 20) + 12_345, ops_per_key=8, n_elems=0, seed=777,
         warm=1),
    # tag passes just past 2^16 keys (runs of 128)
    dict(crdt_type=2, n_dcs=16, n_keys=(1 << 16) + 4_321, ops_per_key=16, n_elems=8, seed=778),
    dict(crdt_type=3, n_dcs=64, n_keys=(1 << 16) + 999, ops_per_key=8, n_elems=4, seed=779,
         warm=1),
]
ORDERS = {"default": {}, "identity": {"AGN_XCD_REMAP": "0"}, "xcd": {"AGN_XCD_REMAP": "1"},
          "runs7": {"AGN_XCD_CHUNK": "7"}, "runs300": {"AGN_XCD_CHUNK": "300"}}


def _equal_all(crdt, got, want, K):
    """Every key's result, vectorised (no error flags in generated logs)."""
    assert np.array_equal(got.flags[:K], want.flags[:K])
    assert np.array_equal(got.count[:K], want.count[:K])
    assert np.array_equal(got.hole[:K], want.hole[:K])
    ct = (want.flags[:K] & _abi.F_CT_IGNORE) == 0
    assert np.array_equal(got.lastct[:K][ct], want.lastct[:K][ct])
    if crdt == _abi.COUNTER_PN:
        assert np.array_equal(got.value[:K], want.value[:K])
        return
    assert np.array_equal(got.out_n[:K], want.out_n[:K])
    assert np.array_equal(got.out_off[:K], want.out_off[:K])
    n = want.out_n[:K].astype(np.int64)
    pos = np.repeat(want.out_off[:K].astype(np.int64), n) + \
        (np.arange(int(n.sum())) - np.repeat(np.cumsum(n) - n, n))
    assert np.array_equal(got.out_tag[pos], want.out_tag[pos])
    assert np.array_equal(got.out_tok[pos], want.out_tok[pos])


@pytest.mark.parametrize("spec", BULK, ids=["counter_cold", "counter_warm", "set_aw", "register_mv_warm"])
def test_bulk_block_orders_all_keys(eng, oracle_lib, monkeypatch, spec):
    """Batches just past the bulk thresholds (counter 2^20 requests, tag passes
    2^16 keys), every key against the oracle under each block order the
    launchers choose from (block_order: identity, XCD-aware, runs of g --
    odd and larger than a super-run's share), the default included."""
    cfg = _abi.AgnGenCfg(**{"key_base": 0, "key_stride": 1, "warm": 0, **spec})
    K, D = cfg.n_keys, cfg.n_dcs
    cap = None if cfg.crdt_type == 1 else \
        np.arange(K + 1, dtype=np.uint64) * np.uint64(cfg.ops_per_key)
    hl, hr = gen_host(cfg)
    want = alloc_result(K, D, sparse=False, cap_off=cap)
    assert oracle_lib.oracle_materialize(C.byref(hl), C.byref(hr),
                                         C.byref(result_struct(want)), 4) == 0
    free_gen_host(hl, hr)
    assert 0.05 < want.count.mean() / cfg.ops_per_key < 0.95
    dl, dr = eng.gen_dev(cfg)
    try:
        for name, env in ORDERS.items():
            for k in ("AGN_XCD_REMAP", "AGN_XCD_CHUNK"):
                monkeypatch.delenv(k, raising=False)
            for k, v in env.items():
                monkeypatch.setenv(k, v)
            res = eng.alloc_result(K, D, sparse=False, cap_off=cap)
            eng.materialize(dl, dr, res)
            eng.sync()
            got = eng.fetch_result(res)
            for b in res.bufs.values():
                b.free()
            try:
                _equal_all(cfg.crdt_type, got, want, K)
            except AssertionError as e:
                raise AssertionError(f"block order {name}") from e
    finally:
        eng.free_gen(dl, dr)


# ------------------------------------------------------------------ GST / base selection
@pytest.mark.parametrize("D,P,E,p_undef,p_absent", [(2, 3, 1, 0.0, 0.0), (8, 64, 4, 0.05, 0.1),
                                                    (256, 4096, 2, 0.0, 0.0),
                                                    (256, 4096, 3, 0.001, 0.02),
                                                    (5, 1000, 7, 0.01, 0.3), (300, 17, 2, 0.1, 0.5)])
def test_gst_vs_oracle(eng, oracle_lib, D, P, E, p_undef, p_absent):
    rng = np.random.default_rng(D * 7 + P)
    clocks = (1_700_000_000_000_000 + rng.integers(0, 10 ** 9, (E, P, D))).astype(np.uint64)
    clocks[rng.random((E, P, D)) < p_absent] = np.uint64(_abi.U64_MAX)
    defined = (rng.random((E, P)) >= p_undef).astype(np.uint8)
    want = np.zeros((E, D + 1), np.uint64)
    oracle_lib.oracle_gst_min(D, P, E, clocks.ctypes.data, defined.ctypes.data, want.ctypes.data, 1)
    dc, dd = eng.upload(clocks), eng.upload(defined)
    out = eng.empty(E * (D + 1) * 8)
    eng.gst_min(D, P, E, dc.ptr, dd.ptr, out.ptr)
    eng.gst_finalize(D, E, out.ptr)
    got = eng.download(out, np.uint64, (E, D + 1))
    assert np.array_equal(got, want)
    for b in (dc, dd, out):
        b.free()


def test_gst_kats_gpu(eng):
    from oracle import py_oracle as po
    for c in kats({"gst"}):
        parts = {p: (po.UNDEFINED if v == "undefined" else to_vc(v)) for p, v in c["parts"].items()}
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
        dc, dd, out = eng.upload(clocks), eng.upload(defined), eng.empty((D + 1) * 8)
        eng.gst_min(D, P, 1, dc.ptr, dd.ptr, out.ptr)
        eng.gst_finalize(D, 1, out.ptr)
        got = eng.download(out, np.uint64, (D + 1,))
        res = {d: int(got[j]) for j, d in enumerate(dcs) if int(got[j]) != _abi.U64_MAX}
        assert res == to_vc(c["expect"]), c["name"]


def test_select_base_vs_oracle(eng, oracle_lib):
    rng = np.random.default_rng(3)
    for D in (2, 8, 64, 130):
        n = 500
        lens = rng.integers(0, 11, n)
        off = np.zeros(n + 1, np.uint64)
        off[1:] = np.cumsum(lens)
        M = int(off[-1])
        clocks = rng.integers(0, 100, (max(M, 1), D)).astype(np.uint64)
        W = (D + 63) // 64
        cm = rng.integers(0, 2 ** 62, (max(M, 1), W)).astype(np.uint64)
        R = rng.integers(50, 150, (n, D)).astype(np.uint64)
        Rm = rng.integers(0, 2 ** 62, (n, W)).astype(np.uint64) | np.uint64(0x5555)
        wi, wf = np.zeros(n, np.int32), np.zeros(n, np.uint8)
        oracle_lib.oracle_select_base(D, n, off.ctypes.data, clocks.ctypes.data, cm.ctypes.data,
                                      R.ctypes.data, Rm.ctypes.data, wi.ctypes.data,
                                      wf.ctypes.data)
        bufs = [eng.upload(x) for x in (off, clocks, cm, R, Rm)]
        oi, of = eng.empty(n * 4), eng.empty(n)
        eng.select_base(D, n, *[b.ptr for b in bufs], oi.ptr, of.ptr)
        assert np.array_equal(eng.download(oi, np.int32, (n,)), wi)
        assert np.array_equal(eng.download(of, np.uint8, (n,)), wf)


def test_rccl_single_rank_min_allreduce(eng):
    from antidote_amd._lib import EngineError
    try:  # the session's context may already hold its single-rank communicator
        eng.comm_init(1, 0, Engine.unique_id())
    except EngineError:
        pass
    v = np.array([5, 3, _abi.U64_MAX, 1], np.uint64)
    b = eng.upload(v)
    eng.gst_allreduce(b.ptr, 4)
    eng.sync()
    assert np.array_equal(eng.download(b, np.uint64, (4,)), v)


@pytest.mark.parametrize("crdt", [_abi.SET_AW, _abi.REGISTER_MV])
def test_tags_state_refs_need_their_arrays(eng, crdt):
    """agn_read.base_value without base_off names AGN_SS_STATE references into
    base_tag / base_tok: with either array missing the call fails with
    AGN_EINVAL before any kernel reads them (not an out-of-bounds read)."""
    from antidote_amd._lib import EngineError
    log, req, cap = random_case(9 + crdt, crdt, 40, 3, 20)
    dl, dr = eng.upload_log(log), eng.upload_read(req, sparse=False)
    refs = eng.empty(8 * req.n_req)
    dr.struct.base_off = None
    dr.struct.base_tag = None
    dr.struct.base_tok = None
    dr.struct.base_value = refs.ptr
    dres = eng.alloc_result(req.n_req, log.n_dcs, sparse=False, cap_off=cap)
    with pytest.raises(EngineError) as ei:
        eng.materialize(dl, dr, dres)
    assert ei.value.code == _abi.EINVAL
