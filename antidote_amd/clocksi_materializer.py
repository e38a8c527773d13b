"""Host mirror of clocksi_materializer (src/clocksi_materializer.erl) over the
C ABI.  Same names, argument meaning and error behaviour:

  new(Type)                                   :41-43
  materialize(Type, TxId, MinSnapshotTime, #snapshot_get_response{}) :82-101
      -> ("ok", Snapshot, NewLastOp, LastOpCt | "ignore", IsNewSS, Count)
       | ("error", {unexpected_operation, Op, Type})
       raises CorruptedOpsCache on a type mismatch (:190-191)
  materialize_eager(Type, Snapshot, Ops)      :272-274

plus materialize_batch(...) — many materialize/4 calls in one launch, the
form the NIF's micro-batching queue uses.  Every filter decision and every
effect application runs in the HIP kernels (agn_materialize); this module
only encodes terms and decodes results.
"""
from __future__ import annotations

from . import _abi
from .encode import IGNORE, ClocksiPayload, DcTable, LogEncoder, ReadEncoder, decode_clock
from .records import (COUNTER_PN, REGISTER_MV, SET_AW, CorruptedOpsCache,
                      MaterializedSnapshot, SnapshotGetResponse, ops_oldest_first)

_TYPE_IDS = {COUNTER_PN: _abi.COUNTER_PN, SET_AW: _abi.SET_AW, REGISTER_MV: _abi.REGISTER_MV}
_engines: dict = {}


def engine(device: int = 0):
    from .engine import Engine
    e = _engines.get(device)
    if e is None:
        e = _engines[device] = Engine(device)
    return e


def type_id(typ: str) -> int:
    try:
        return _TYPE_IDS[typ]
    except KeyError:
        raise ValueError(("undef", typ)) from None  # Type:new() of an unknown module


def new(typ: str):
    """materializer:create_snapshot/1 = Type:new()."""
    type_id(typ)
    return 0 if typ == COUNTER_PN else []


def value(typ: str, state):
    """Type:value/1."""
    if typ == COUNTER_PN:
        return state
    if typ == SET_AW:
        return [e for e, _ in state]
    return [v for v, _ in state]


def _n_dcs(clocks) -> int:
    dcs = set()
    for c in clocks:
        if isinstance(c, dict):
            dcs |= set(c)
    return max(1, len(dcs))


def _base_pairs(typ, snapshot):
    if typ == COUNTER_PN:
        return snapshot
    if typ == SET_AW:
        return [(e, list(toks)) for e, toks in snapshot]
    return [(v, t) for v, t in snapshot]


def _decode_state(typ, enc, res, i):
    o, n = int(res.out_off[i]), int(res.out_n[i])
    pairs = [(enc.tags.term(int(t)), enc.tokens.term(int(k)))
             for t, k in zip(res.out_tag[o:o + n], res.out_tok[o:o + n])]
    if typ == SET_AW:
        st: dict = {}
        for e, tk in pairs:           # device order: elem id, then add order
            st.setdefault(e, []).append(tk)
        return sorted(st.items(), key=lambda kv: kv[0])   # orddict by elem term
    return sorted(pairs)              # insert_sorted({Value, Token})


def materialize_batch(typ: str, reads, device: int = 0):
    """reads: [(TxId, MinSnapshotTime, SnapshotGetResponse)] -> list of
    materialize/4 results (CorruptedOpsCache instances are returned, not
    raised, so one bad key does not hide the others)."""
    tid = type_id(typ)
    resp_clocks = []
    for _tx, r, resp in reads:
        resp_clocks.append(r)
        if isinstance(resp.snapshot_time, dict):
            resp_clocks.append(resp.snapshot_time)
        for _i, p in ops_oldest_first(resp.ops_list):
            resp_clocks.append(p.snapshot_time)
            resp_clocks.append({p.commit_time[0]: p.commit_time[1]})
    D = _n_dcs(resp_clocks)
    enc = LogEncoder(tid, D, dcs=DcTable())
    rd = ReadEncoder(enc, tid)
    for txid, R, resp in reads:
        k = enc.add_key([(i, ClocksiPayload(p.key, p.type, p.op_param, p.snapshot_time,
                                            p.commit_time, p.txid))
                         for i, p in ops_oldest_first(resp.ops_list)])
        rd.add(k, R, resp.snapshot_time, txid,
               _base_pairs(typ, resp.materialized_snapshot.value))
    log = enc.build()
    req = rd.build()
    cap = None
    if tid != _abi.COUNTER_PN:
        from .encode import state_capacity
        cap = state_capacity(log, req)
    res = engine(device).materialize_host(log, req, sparse=True, cap_off=cap)
    out = []
    for i in range(req.n_req):
        f = int(res.flags[i])
        if f & _abi.F_ERR_CORRUPTED:
            out.append(CorruptedOpsCache())
            continue
        if f & _abi.F_ERR_UNEXPECTED:
            e = int(res.err_pos[i])
            out.append(("error", ("unexpected_operation", log.invalid_terms.get(e), typ)))
            continue
        if f & _abi.F_ERR_CAPACITY:
            raise RuntimeError("materialize: live state exceeds the device table capacity")
        ct = IGNORE if f & _abi.F_CT_IGNORE else decode_clock(res.lastct[i], res.lastct_mask[i],
                                                               enc.dcs)
        val = int(res.value[i]) if tid == _abi.COUNTER_PN else _decode_state(typ, enc, res, i)
        out.append(("ok", val, int(res.hole[i]), ct, bool(f & _abi.F_NEWSS), int(res.count[i])))
    return out


def materialize(typ: str, txid, min_snapshot_time: dict, resp: SnapshotGetResponse,
                device: int = 0):
    r = materialize_batch(typ, [(txid, min_snapshot_time, resp)], device)[0]
    if isinstance(r, CorruptedOpsCache):
        raise r
    return r


def materialize_eager(typ: str, snapshot, effects, device: int = 0):
    """Apply effects in order without checks (materializer:materialize_eager/3):
    one key whose ops are all inside the read snapshot."""
    ops = [(i + 1, ClocksiPayload("eager", typ, e, {"eager": 2 * i}, ("eager", 2 * i + 1), None))
           for i, e in enumerate(effects)]
    resp = SnapshotGetResponse(ops[::-1], len(ops), MaterializedSnapshot(0, snapshot), IGNORE,
                               True)
    r = materialize(typ, IGNORE, {"eager": 2 * len(effects) + 1}, resp, device)
    return r if r[0] == "error" else r[1]
