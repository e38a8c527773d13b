"""Cross-check the two independent restatements of the reference on random
inputs: oracle/oracle.c (SoA, the GPU parity checker) and oracle/py_oracle.py
(dict clocks, literal transcription of the Erlang).  Covers sparse clocks,
warm reads, TxId matches, invalid effects, corrupted keys, multi-entry ops and
base states for all three CRDT types."""
import ctypes as C

import numpy as np
import pytest

from antidote_amd import _abi
from antidote_amd.encode import alloc_result, log_struct, read_struct, result_struct
from oracle import py_oracle as po
from synth import random_case

TYPES = {_abi.COUNTER_PN: po.COUNTER_PN, _abi.SET_AW: po.SET_AW,
         _abi.REGISTER_MV: po.REGISTER_MV}


def present(mask_row, d):
    return mask_row is None or (int(mask_row[d >> 6]) >> (d & 63)) & 1


def to_dict(vals, mask_row, D):
    return {d: int(vals[d]) for d in range(D) if present(mask_row, d)}


def key_ops(log, k, typ):
    """SoA key -> ops list newest-first [(op_id, Payload)] + entry->op index."""
    D = log.n_dcs
    a, b = int(log.key_off[k]), int(log.key_off[k + 1])
    groups = []
    for e in range(a, b):
        if groups and log.op_id[e] == log.op_id[e - 1] and e > a:
            groups[-1].append(e)
        else:
            groups.append([e])
    ops = []
    for g in groups:
        e0 = g[0]
        oc = to_dict(log.oc[e0], None if log.oc_mask is None else log.oc_mask[e0], D)
        dc = next(iter(oc))
        if log.crdt_type == _abi.COUNTER_PN:
            v = int(log.eff[e0])
            eff = ("invalid",) if v == _abi.EFFECT_INVALID else v
        elif any(int(log.tag[e]) == _abi.TAG_INVALID for e in g):
            eff = ("invalid",)
        else:
            ro = log.rem_off
            parts = []
            for e in g:
                rems = [int(x) for x in log.rem_tok[int(ro[e]):int(ro[e + 1])]]
                add = int(log.add_tok[e])
                if log.crdt_type == _abi.SET_AW:
                    parts.append((int(log.tag[e]), [add] if add else [], rems))
                else:
                    parts.append(("reset", rems) if add == 0 else (int(log.tag[e]), add, rems))
            eff = parts if log.crdt_type == _abi.SET_AW else parts[0]
        ops.append((int(log.op_id[e0]), po.Payload("k", typ, eff, oc, (dc, oc[dc]),
                                                   int(log.txid[e0]))))
    if log.key_type[k] == _abi.TYPE_MIXED and ops:
        last = ops[-1][1]
        ops[-1] = (ops[-1][0], po.Payload("k", "other_type", last.op_param, last.snapshot_time,
                                          last.commit_time, last.txid))
    return ops[::-1]


def py_run(log, req, i):
    typ = TYPES[log.crdt_type]
    D = log.n_dcs
    k = int(req.keys[i])
    ops = key_ops(log, k, typ)
    R = to_dict(req.R[i], req.R_mask[i] if SPARSE[0] else None, D)
    sct = po.IGNORE if req.sct_ignore[i] else \
        to_dict(req.sct[i], req.sct_mask[i] if SPARSE[0] else None, D)
    txid = po.IGNORE if int(req.txid[i]) == 0 else int(req.txid[i])
    if log.crdt_type == _abi.COUNTER_PN:
        base = int(req.base_value[i])
    else:
        pairs = [(int(t), int(x)) for t, x in zip(req.base_tag[int(req.base_off[i]):
                                                               int(req.base_off[i + 1])],
                                                  req.base_tok[int(req.base_off[i]):
                                                               int(req.base_off[i + 1])])]
        if log.crdt_type == _abi.SET_AW:
            st: dict = {}
            for t, x in pairs:
                st.setdefault(t, []).append(x)
            base = sorted(st.items())
        else:
            base = pairs
    resp = po.SnapshotGetResponse(ops, len(ops), po.MaterializedSnapshot(0, base), sct, True)
    try:
        return po.materialize(typ, txid, R, resp)
    except po.CorruptedOpsCache:
        return ("raise",)


SPARSE = [False]


def c_decode(log, req, res, i, sparse):
    f = int(res.flags[i])
    if f & _abi.F_ERR_CORRUPTED:
        return ("raise",)
    if f & _abi.F_ERR_UNEXPECTED:
        return ("error", int(res.err_pos[i]))
    D = log.n_dcs
    ct = po.IGNORE if f & _abi.F_CT_IGNORE else \
        to_dict(res.lastct[i], res.lastct_mask[i] if sparse else None, D)
    if log.crdt_type == _abi.COUNTER_PN:
        val = int(res.value[i])
    else:
        o, n = int(res.out_off[i]), int(res.out_n[i])
        pairs = [(int(t), int(x)) for t, x in zip(res.out_tag[o:o + n], res.out_tok[o:o + n])]
        if log.crdt_type == _abi.SET_AW:
            st: dict = {}
            for t, x in pairs:
                st.setdefault(t, []).append(x)
            val = sorted(st.items())
        else:
            val = pairs
    return ("ok", val, int(res.hole[i]), ct, bool(f & _abi.F_NEWSS), int(res.count[i]))


CASES = []
for crdt in (_abi.COUNTER_PN, _abi.SET_AW, _abi.REGISTER_MV):
    for D in (1, 3, 8, 17):
        for sparse in (False, True):
            CASES.append((crdt, D, sparse))


@pytest.mark.parametrize("crdt,D,sparse", CASES)
def test_c_oracle_matches_py_oracle(oracle_lib, crdt, D, sparse):
    SPARSE[0] = sparse
    log, req, cap = random_case(1000 * crdt + 10 * D + sparse, crdt, 40, D, 12, sparse=sparse,
                                warm=0.4, txid=0.3, invalid=0.03, corrupt=0.05,
                                multi=0.2 if crdt == _abi.SET_AW else 0.0, base=0.5,
                                identity=False)
    res = alloc_result(req.n_req, D, sparse=True, cap_off=cap)
    ls, rs, os_ = log_struct(log), read_struct(req, sparse=sparse), result_struct(res)
    assert oracle_lib.oracle_materialize(C.byref(ls), C.byref(rs), C.byref(os_), 2) == 0
    for i in range(req.n_req):
        py = py_run(log, req, i)
        c = c_decode(log, req, res, i, True)
        if py[0] == "error":
            assert c[0] == "error", (i, py, c)
            # the failing op is the same op
            k = int(req.keys[i])
            e = c[1]
            assert int(log.key_off[k]) <= e < int(log.key_off[k + 1])
            assert py[1][1] == ("invalid",)
            continue
        assert c == py, (i, c, py)
