"""CPU checks of the C-ABI boundary: the library loads, exports exactly what
include/antidote_gpu.h declares, the ctypes mirror has the C struct layout,
and the host-only entry points (no GPU needed) behave."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

from antidote_amd import _abi
from antidote_amd._lib import LIB_PATH, load
from antidote_amd.encode import alloc_result, result_struct, state_capacity
from oracle import py_oracle as po

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "antidote_gpu.h")


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "antidote_amd", "csrc")])
    return load()


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"^\s*(?:int|const char \*)\s*(agn_\w+)\s*\(", src, flags=re.M))


def test_exports_match_header(lib):
    want = header_functions()
    assert want == set(_abi.PROTOTYPES), want ^ set(_abi.PROTOTYPES)
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB_PATH], text=True)
    exported = {ln.split()[-1] for ln in out.splitlines() if " T agn_" in ln}
    assert want <= exported, want - exported
    for name in want:
        assert getattr(lib, name) is not None


def test_struct_layout_matches_c():
    prog = r'''
#include <stdio.h>
#include <stddef.h>
#include "antidote_gpu.h"
#define F(T, m) printf("%s.%s %zu\n", #T, #m, offsetof(T, m));
int main(void) {
  printf("agn_log %zu\nagn_read %zu\nagn_result %zu\nagn_gen_cfg %zu\n", sizeof(agn_log),
         sizeof(agn_read), sizeof(agn_result), sizeof(agn_gen_cfg));
  F(agn_log, rem_tok) F(agn_log, eff) F(agn_log, key_id0) F(agn_log, key_mask)
  F(agn_read, req_type) F(agn_read, base_tok)
  F(agn_result, out_tok) F(agn_result, err_pos) F(agn_gen_cfg, warm) F(agn_gen_cfg, key_stride)
  return 0; }
'''
    with tempfile.TemporaryDirectory() as d:
        c, exe = os.path.join(d, "l.c"), os.path.join(d, "l")
        open(c, "w").write(prog)
        subprocess.check_call(["gcc", "-I", os.path.dirname(HEADER), c, "-o", exe])
        got = dict(ln.rsplit(" ", 1) for ln in subprocess.check_output([exe], text=True).splitlines())
    py = {"agn_log": _abi.AgnLog, "agn_read": _abi.AgnRead, "agn_result": _abi.AgnResult,
          "agn_gen_cfg": _abi.AgnGenCfg}
    for k, v in got.items():
        if "." in k:
            t, m = k.split(".")
            assert getattr(py[t], m).offset == int(v), k
        else:
            assert C.sizeof(py[k]) == int(v), k


def test_open_without_gpu_fails_loudly(lib):
    n = C.c_int(-1)
    assert lib.agn_device_count(C.byref(n)) == 0
    if n.value > 0:
        pytest.skip("a GPU is visible")
    ctx = C.c_void_p()
    assert lib.agn_open(0, C.byref(ctx)) == _abi.ENODEV
    assert lib.agn_last_error()
    from antidote_amd._lib import EngineUnavailable
    from antidote_amd.engine import Engine
    with pytest.raises(EngineUnavailable):
        Engine(0)


def test_null_arguments_are_einval(lib):
    assert lib.agn_materialize(None, None, None, None, None) == _abi.EINVAL
    assert lib.agn_update_stable(3, None, None, None) == _abi.EINVAL
    assert lib.agn_strerror(_abi.EINVAL) == b"invalid argument"


def test_update_stable_matches_reference(lib):
    rng = np.random.default_rng(0)
    for _ in range(200):
        D = int(rng.integers(1, 6))
        last = rng.integers(0, 10, D).astype(np.uint64)
        new = rng.integers(0, 10, D).astype(np.uint64)
        last[rng.random(D) < 0.3] = np.uint64(_abi.U64_MAX)
        new[rng.random(D) < 0.3] = np.uint64(_abi.U64_MAX)
        ld = {d: int(v) for d, v in enumerate(last) if v != _abi.U64_MAX}
        nd = {d: int(v) for d, v in enumerate(new) if v != _abi.U64_MAX}
        ch_ref, acc = po.update_stable(ld, nd)
        ch = C.c_int(0)
        assert lib.agn_update_stable(D, last.ctypes.data, new.ctypes.data, C.byref(ch)) == 0
        got = {d: int(v) for d, v in enumerate(last) if v != _abi.U64_MAX}
        assert got == acc and bool(ch.value) == ch_ref


def test_state_capacity_matches_encoder(lib):
    from synth import random_case
    from antidote_amd.encode import log_struct, read_struct
    log, req, cap = random_case(4, _abi.SET_AW, 50, 4, 20, base=0.5)
    got = np.zeros(req.n_req + 1, np.uint64)
    assert lib.agn_state_capacity(C.byref(log_struct(log)), C.byref(read_struct(req)),
                                  got.ctypes.data) == 0
    assert np.array_equal(got, cap)


def test_host_generator_deterministic_and_shaped(lib, oracle_lib):
    from antidote_amd.engine import free_gen_host, gen_host, host_view
    for crdt, D, N, E in ((1, 8, 64, 0), (2, 16, 256, 32), (3, 64, 100, 16)):
        cfg = _abi.AgnGenCfg(crdt_type=crdt, n_dcs=D, n_keys=300, ops_per_key=N, n_elems=E,
                             seed=20250112 + crdt, key_base=0, key_stride=1)
        a_log, a_req = gen_host(cfg)
        b_log, b_req = gen_host(cfg)
        try:
            K = 300
            oc_a = host_view(a_log.oc, np.uint64, K * N * D).reshape(K, N, D)
            oc_b = host_view(b_log.oc, np.uint64, K * N * D).reshape(K, N, D)
            assert np.array_equal(oc_a, oc_b)
            assert (oc_a > 1_600_000_000_000_000).all()
            # the commit DC's entry grows along each key's log
            assert np.all(np.diff(oc_a.max(axis=2).astype(np.int64), axis=1) > -6000)
            ids = host_view(a_log.op_id, np.uint32, K * N).reshape(K, N)
            assert (ids == np.arange(1, N + 1)).all()
            # a sub-range of keys regenerates identically (per-key streams)
            c2 = _abi.AgnGenCfg(crdt_type=crdt, n_dcs=D, n_keys=10, ops_per_key=N, n_elems=E,
                                seed=cfg.seed, key_base=100, key_stride=1)
            s_log, s_req = gen_host(c2)
            assert np.array_equal(host_view(s_log.oc, np.uint64, 10 * N * D).reshape(10, N, D),
                                  oc_a[100:110])
            free_gen_host(s_log, s_req)
            cap = np.arange(K + 1, dtype=np.uint64) * np.uint64(N) if crdt != 1 else None
            r = alloc_result(K, D, sparse=False, cap_off=cap)
            assert oracle_lib.oracle_materialize(C.byref(a_log), C.byref(a_req),
                                                 C.byref(result_struct(r)), 2) == 0
            frac = r.count.mean() / N
            assert 0.2 < frac < 0.95, frac
            assert not (r.flags & (_abi.F_ERR_CAPACITY | _abi.F_ERR_UNEXPECTED)).any()
        finally:
            free_gen_host(a_log, a_req)
            free_gen_host(b_log, b_req)


def test_descriptors_validate_without_gpu(lib):
    """Every descriptor the tests and the mirror build passes agn_* validation
    (checked before the device is touched: a NULL context is the only error)."""
    import kat_util
    from synth import random_case
    from antidote_amd.encode import log_struct, read_struct
    cases = []
    for crdt in (_abi.COUNTER_PN, _abi.SET_AW, _abi.REGISTER_MV):
        cases.append(random_case(3, crdt, 20, 5, 8, base=0.5))
        cases.append(random_case(4, crdt, 5, 3, 0, empty=1.0))
    for log, req, cap in cases:
        res = alloc_result(req.n_req, log.n_dcs, sparse=True, cap_off=cap)
        rc = lib.agn_materialize_host(None, C.byref(log_struct(log)), C.byref(read_struct(req)),
                                      C.byref(result_struct(res)))
        assert rc == _abi.EINVAL and lib.agn_last_error() == b"null context"
    for c in kat_util.kats({"system_seq"}):
        ops, reads, _ = kat_util.system_seq_log(c)
        run = kat_util.OneKeyRun(c["type"], ops, 1)
        run.add_read(reads[0])

        def fn(ls, rs, os_):
            rc = lib.agn_materialize_host(None, C.byref(ls), C.byref(rs), C.byref(os_))
            assert lib.agn_last_error() == b"null context", lib.agn_last_error()
            return 0
        run.run(fn)


def test_read_cached_validates_without_gpu(lib):
    """agn_read_cached's argument checks run before the device is touched:
    counter_pn with dense clocks and D <= 8 only (ENOTSUP otherwise), the
    cache and log must agree on keys and DCs, an empty batch is a no-op, and
    a valid batch then needs the context."""
    from synth import random_case
    from antidote_amd.encode import log_struct

    def case(crdt, D, sparse=False):
        log, _req, _ = random_case(5, crdt, 12, D, 6, sparse=sparse)
        ls = log_struct(log)
        if log.oc_mask is None:
            ls.oc_mask = None
        c = _abi.AgnSsCache()
        c.n_dcs, c.slots, c.n_keys = D, _abi.SNAPSHOT_THRESHOLD, 12
        bufs = [np.zeros(12, np.uint32), np.zeros(12 * 10 * D, np.uint64),
                np.zeros(12 * 10, np.int64), np.zeros(12 * 10, np.int64)]
        c.n, c.clock, c.last_op, c.value = (b.ctypes.data for b in bufs)
        res = alloc_result(4, D, sparse=False)
        return ls, c, result_struct(res), (log, bufs, res)

    keys = np.arange(4, dtype=np.uint64)
    R = np.zeros((4, 8), np.uint64)
    st, pr, thr = np.zeros(4, np.uint8), np.zeros(4, np.uint8), np.zeros(12 * 8, np.uint64)

    def call(ls, c, os_, n=4):
        return lib.agn_read_cached(None, C.byref(c) if c is not None else None, C.byref(ls), n,
                                   keys.ctypes.data, R.ctypes.data, None, None, C.byref(os_),
                                   st.ctypes.data, pr.ctypes.data, thr.ctypes.data, None)

    ls, c, os_, keep = case(_abi.COUNTER_PN, 8)
    assert call(ls, None, os_) == _abi.EINVAL
    assert call(ls, c, os_, n=0) == _abi.OK
    assert call(ls, c, os_) == _abi.EINVAL and lib.agn_last_error() == b"null context"
    c.n_keys = 11
    assert call(ls, c, os_) == _abi.EINVAL
    for crdt, D, sparse in ((_abi.SET_AW, 4, False), (_abi.COUNTER_PN, 9, False),
                            (_abi.COUNTER_PN, 4, True)):
        ls, c, os_, keep = case(crdt, D, sparse)
        assert call(ls, c, os_) == _abi.ENOTSUP, (crdt, D, sparse)
