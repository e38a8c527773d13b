"""the causal-dependency check of
inter_dc_dep_vnode:try_store/2 and the gentlerain scalar GST of
dc_utilities (get_scalar_stable_time/0, gr branch of get_stable_snapshot/0).

The reference has no unit tests for either (only multi-DC system suites that
cannot run here), so these are pinned by restatement: the C oracle is checked
against the literal dict transcription in oracle/py_oracle.py, and the GPU
kernels against the C oracle bit-exactly."""
import ctypes as C

import numpy as np
import pytest

from antidote_amd import _abi
from oracle import py_oracle as po

U64 = _abi.U64_MAX


def _masks(rng, n, D, p_absent):
    W = (D + 63) // 64
    pres = rng.random((n, D)) >= p_absent
    m = np.zeros((n, W), np.uint64)
    for d in range(D):
        m[:, d >> 6] |= pres[:, d].astype(np.uint64) << np.uint64(d & 63)
    return m, pres


def dep_case(seed, D, n, P, sparse):
    rng = np.random.default_rng(seed)
    pc = rng.integers(1000, 2000, (P, D)).astype(np.uint64)
    part = rng.integers(0, P, n).astype(np.uint32)
    origin = rng.integers(0, D, n).astype(np.uint32)
    # deps at or below the partition clock; half the transactions get one DC
    # ahead of it (which may be the origin DC, whose entry does not count)
    deps = (pc[part] - rng.integers(0, 40, (n, D))).astype(np.uint64)
    ahead = rng.random(n) < 0.5
    col = rng.integers(0, D, n)
    deps[ahead, col[ahead]] = pc[part[ahead], col[ahead]] + np.uint64(1)
    dm = pm = None
    if sparse:
        # a transaction's snapshot mostly names DCs the partition knows; 10 %
        # name one it does not (missing there = 0, so not applicable)
        pm, _ = _masks(rng, P, D, 0.2)
        dm, _ = _masks(rng, n, D, 0.3)
        dm &= pm[part]
        extra = rng.random(n) < 0.1
        xc = rng.integers(0, D, n)
        for t in np.nonzero(extra)[0]:
            dm[t, xc[t] >> 6] |= np.uint64(1 << int(xc[t] & 63))
    return deps, dm, origin, part, pc, pm


def ptr(a):
    return None if a is None else a.ctypes.data


def dep_oracle(lib, D, deps, dm, origin, part, pc, pm):
    ok = np.zeros(len(origin), np.uint8)
    rc = lib.oracle_dep_check(D, len(origin), ptr(deps), ptr(dm), ptr(origin), ptr(part),
                              pc.shape[0], ptr(pc), ptr(pm), ptr(ok))
    assert rc == 0
    return ok


def as_dict(row, mrow, D):
    return {d: int(row[d]) for d in range(D)
            if mrow is None or (int(mrow[d >> 6]) >> (d & 63)) & 1}


@pytest.mark.parametrize("D,sparse", [(1, False), (3, True), (8, False), (64, True), (130, True)])
def test_dep_check_oracle_vs_dict_restatement(oracle_lib, D, sparse):
    deps, dm, origin, part, pc, pm = dep_case(D * 11 + sparse, D, 300, 7, sparse)
    got = dep_oracle(oracle_lib, D, deps, dm, origin, part, pc, pm)
    for t in range(len(origin)):
        want = po.dependencies_satisfied(
            int(origin[t]), as_dict(deps[t], None if dm is None else dm[t], D),
            as_dict(pc[part[t]], None if pm is None else pm[part[t]], D))
        assert bool(got[t]) == want, t
    if D > 1:  # with one DC the origin entry is the only one: always applicable
        assert 0 < got.mean() < 1


def test_dep_check_origin_entry_ignored(oracle_lib):
    """The originating DC's entry is set to 0 on both sides: a transaction far
    ahead in its own DC is still applicable (delivery is in order per DC)."""
    D = 3
    pc = np.array([[10, 10, 10]], np.uint64)
    deps = np.array([[99, 10, 10], [99, 11, 10]], np.uint64)
    ok = dep_oracle(oracle_lib, D, deps, None, np.array([0, 0], np.uint32),
                    np.zeros(2, np.uint32), pc, None)
    assert ok.tolist() == [1, 0]


def gst_case(seed, D, E, p_absent):
    rng = np.random.default_rng(seed)
    v = np.zeros((E, D + 1), np.uint64)
    v[:, :D] = 1_700_000_000_000_000 + rng.integers(0, 10 ** 6, (E, D))
    v[:, :D][rng.random((E, D)) < p_absent] = U64
    v[:, D] = 1
    return v


@pytest.mark.parametrize("D,p_absent", [(1, 0.0), (5, 0.3), (256, 0.0), (300, 0.5), (4, 1.0)])
def test_gst_scalar_oracle_vs_dict_restatement(oracle_lib, D, p_absent):
    v = gst_case(D, D, 9, p_absent)
    want_rows = [po.scalar_stable_time({d: int(r[d]) for d in range(D) if r[d] != U64})
                 for r in v]
    out = np.zeros(9, np.uint64)
    assert oracle_lib.oracle_gst_scalar(D, 9, ptr(v), ptr(out)) == 0
    for e in range(9):
        got = {d: int(v[e, d]) for d in range(D) if v[e, d] != U64}
        assert got == want_rows[e]
        assert (int(out[e]) == U64) == (not want_rows[e])
        if want_rows[e]:
            assert int(out[e]) == min(want_rows[e].values())


# ------------------------------------------------------------------ GPU parity
@pytest.mark.gpu
@pytest.mark.parametrize("D,sparse,n", [(1, False, 10), (3, True, 1000), (8, False, 5000),
                                        (64, True, 3000), (256, False, 2000),
                                        (300, True, 500)])
def test_dep_check_gpu_vs_oracle(eng, oracle_lib, D, sparse, n):
    deps, dm, origin, part, pc, pm = dep_case(D * 13 + n, D, n, 16, sparse)
    want = dep_oracle(oracle_lib, D, deps, dm, origin, part, pc, pm)
    bufs = [eng.upload(x) if x is not None else None for x in (deps, dm, origin, part, pc, pm)]
    out = eng.empty(n)
    eng.dep_check(D, n, *[b.ptr if b is not None else None for b in bufs[:4]], pc.shape[0],
                  bufs[4].ptr, bufs[5].ptr if bufs[5] is not None else None, out.ptr)
    got = eng.download(out, np.uint8, (n,))
    assert np.array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("D,sparse,n,P", [(8, False, 300_000, 5000), (5, True, 123_457, 3),
                                          (64, True, 70_001, 100), (16, False, 99_999, 1)])
def test_dep_check_gpu_bulk_vs_oracle(eng, oracle_lib, D, sparse, n, P):
    """The resident-grid kernel at bulk size: many tiles per wave (4 per step),
    ragged tails, partition clocks staged in LDS (P x D words <= 48 KB) or read
    from memory (P = 5000 at D = 8: 320 KB)."""
    deps, dm, origin, part, pc, pm = dep_case(D * 17 + n, D, n, P, sparse)
    want = dep_oracle(oracle_lib, D, deps, dm, origin, part, pc, pm)
    assert 0 < want.mean() < 1
    bufs = [eng.upload(x) if x is not None else None for x in (deps, dm, origin, part, pc, pm)]
    out = eng.empty(n)
    eng.dep_check(D, n, *[b.ptr if b is not None else None for b in bufs[:4]], pc.shape[0],
                  bufs[4].ptr, bufs[5].ptr if bufs[5] is not None else None, out.ptr)
    assert np.array_equal(eng.download(out, np.uint8, (n,)), want)


@pytest.mark.gpu
@pytest.mark.parametrize("D,E,p_absent", [(1, 3, 0.0), (5, 100, 0.3), (256, 256, 0.0),
                                          (300, 17, 0.5), (4, 8, 1.0)])
def test_gst_scalar_gpu_vs_oracle(eng, oracle_lib, D, E, p_absent):
    v = gst_case(D + E, D, E, p_absent)
    want, wg = v.copy(), np.zeros(E, np.uint64)
    oracle_lib.oracle_gst_scalar(D, E, ptr(want), ptr(wg))
    dv, dg = eng.upload(v), eng.empty(E * 8)
    eng.gst_scalar(D, E, dv.ptr, dg.ptr)
    assert np.array_equal(eng.download(dv, np.uint64, (E, D + 1)), want)
    assert np.array_equal(eng.download(dg, np.uint64, (E,)), wg)
