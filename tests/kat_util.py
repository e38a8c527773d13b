"""Helpers turning tests/golden/kats.json cases into oracle / engine inputs."""
from __future__ import annotations

import json
import os

import numpy as np

from antidote_amd import _abi
from antidote_amd.encode import (ClocksiPayload, DcTable, LogEncoder, ReadEncoder,
                                  alloc_result, decode_clock, log_struct, read_struct,
                                  result_struct, state_capacity)
from oracle import py_oracle as po

HERE = os.path.dirname(os.path.abspath(__file__))
TYPES = {"counter_pn": po.COUNTER_PN, "set_aw": po.SET_AW, "register_mv": po.REGISTER_MV}


def load_kats():
    with open(os.path.join(HERE, "golden", "kats.json")) as f:
        return json.load(f)["cases"]


def kats(kind):
    return [c for c in load_kats() if c["kind"] in kind]


def to_vc(pairs):
    if pairs is None:
        return po.IGNORE
    return {(tuple(d) if isinstance(d, list) else d): t for d, t in pairs}


def effect_of(p):
    e = p["p"]
    if isinstance(e, dict) and "invalid" in e:
        return ("invalid_term", e["invalid"])
    if isinstance(e, list):
        return tuple(e)
    return e


def to_payload(p, typ):
    return po.Payload(key="k", type=typ, op_param=effect_of(p), snapshot_time=to_vc(p["ss"]),
                      commit_time=tuple(p["ct"]), txid=p["tx"])


def py_ops(case):
    typ = TYPES[case["type"]]
    return [(i, to_payload(p, typ)) for i, p in case["ops"]]


# ------------------------------------------------------------ C-oracle / engine path
def n_dcs_of(*clocks):
    dcs = set()
    for c in clocks:
        if isinstance(c, dict):
            dcs |= set(c)
    return max(1, len(dcs))


class OneKeyRun:
    """Encode one key's ops (newest-first list, like #snapshot_get_response.ops_list)
    and a list of reads against it into SoA arrays."""

    def __init__(self, typ_name, ops_newest_first, n_dcs, dense=False):
        self.typ = _abi.TYPE_IDS[TYPES.get(typ_name, typ_name)]
        self.enc = LogEncoder(self.typ, n_dcs, dense=dense)
        oldest_first = list(reversed(ops_newest_first))
        payloads = [(i, ClocksiPayload(p.key, p.type, p.op_param, p.snapshot_time,
                                       p.commit_time, p.txid)) for i, p in oldest_first]
        self.enc.add_key(payloads)
        self.log = self.enc.build()
        self.reads = ReadEncoder(self.enc)

    def add_read(self, R, sct=po.IGNORE, txid=po.IGNORE, base=None):
        self.reads.add(0, R, sct, txid, base)

    def run(self, materialize_fn):
        """materialize_fn(log_struct, read_struct, result_struct) -> int"""
        req = self.reads.build()
        cap = state_capacity(self.log, req) if self.typ != _abi.COUNTER_PN else None
        res = alloc_result(req.n_req, self.log.n_dcs, sparse=True, cap_off=cap)
        ls, rs, os_ = log_struct(self.log), read_struct(req), result_struct(res)
        rc = materialize_fn(ls, rs, os_)
        assert rc == 0, rc
        return req, res

    def decode(self, res, i):
        """-> ("ok", value, hole, ct, newss, count) | ("error", ...) like materialize/4."""
        f = int(res.flags[i])
        if f & _abi.F_ERR_CORRUPTED:
            return ("raise", "corrupted_ops_cache")
        if f & _abi.F_ERR_UNEXPECTED:
            e = int(res.err_pos[i])
            return ("error", ("unexpected_operation", self.log.invalid_terms.get(e), self.typ))
        ct = po.IGNORE if f & _abi.F_CT_IGNORE else decode_clock(res.lastct[i], res.lastct_mask[i],
                                                                  self.enc.dcs)
        if self.typ == _abi.COUNTER_PN:
            val = int(res.value[i])
        else:
            o, n = int(res.out_off[i]), int(res.out_n[i])
            pairs = [(self.enc.tags.term(int(t)), self.enc.tokens.term(int(k)))
                     for t, k in zip(res.out_tag[o:o + n], res.out_tok[o:o + n])]
            if self.typ == _abi.SET_AW:
                st = {}
                for e, tk in pairs:
                    st.setdefault(e, []).append(tk)
                val = sorted(st.items(), key=lambda kv: kv[0])
            else:
                val = sorted(pairs)
        return ("ok", val, int(res.hole[i]), ct, bool(f & _abi.F_NEWSS), int(res.count[i]))


def oracle_fn(lib):
    import ctypes as C

    def fn(ls, rs, os_):
        return lib.oracle_materialize(C.byref(ls), C.byref(rs), C.byref(os_), 1)
    return fn


# ------------------------------------------------------------ downstream (system KATs)
class Downstream:
    """antidote_crdt downstream/2 restated for the system-test KATs (set_aw
    add/remove, register_mv assign): the effect observes the current state."""

    def __init__(self, typ):
        self.typ = typ
        self.n = 0

    def token(self):
        self.n += 1
        return f"tok{self.n}".encode()

    def effect(self, state, upd):
        op, arg = upd
        if self.typ == po.COUNTER_PN:
            # antidote_crdt_counter_pn downstream: increment N -> N, decrement N -> -N
            return {"increment": arg, "decrement": -arg}[op]
        if self.typ == po.SET_AW:
            # add / remove carry one element, add_all / remove_all a list; the
            # effect is one {Elem, AddTokens, ObservedTokens} part per distinct
            # element, sorted by element
            elems = sorted(set(arg)) if op in ("add_all", "remove_all") else [arg]
            cur = dict(state)
            adding = op in ("add", "add_all")
            return [(e, [self.token()] if adding else [], list(cur.get(e, [])))
                    for e in elems]
        if self.typ == po.REGISTER_MV:
            if op == "reset":   # map_rr remove of an embedded register_mv
                return ("reset", [t for _, t in state])
            return (arg, self.token(), [t for _, t in state])
        raise ValueError(op)


def system_seq_log(case):
    """Sequential single-DC log for a system_seq KAT: op i commits at 10*(i+1),
    snapshot = previous commit.  Returns (ops newest-first, read clocks)."""
    typ = TYPES[case["type"]]
    ds = Downstream(typ)
    state = po.crdt_new(typ)
    ops, reads = [], []
    for i, upd in enumerate(case["updates"]):
        eff = ds.effect(state, upd)
        state = po.crdt_update(typ, eff, state)
        p = po.Payload("k", typ, eff, {"dc1": 10 * i}, ("dc1", 10 * (i + 1)), i + 1)
        ops.insert(0, (i + 1, p))
        reads.append({"dc1": 10 * (i + 1)})
    return ops, reads, state


def system_txn_log(case):
    """Multi-DC transaction history of a system_txn KAT -> per-key op logs
    (newest-first, like #snapshot_get_response.ops_list) and the reads.

    Clock model (Clock-SI, SURVEY.md §3 call stacks 2/3): transaction i runs at
    its DC x with snapshot ss = max(commit VCs of its dependencies) with
    ss[x] = "now" = 10(i+1) - 5 (so it sees every earlier local commit), and
    commits at (x, 10(i+1)); its commit VC is ss with x := 10(i+1).  All its
    updates share the txid and commit time, and each update's effect observes
    the state left by the transaction's earlier updates (read-your-writes of
    the interactive coordinator).  A read "at" a list of transactions uses
    the max of their commit VCs, i.e. check_read_key(..., CommitTime, static)."""
    typ = TYPES[case["type"]]
    ds = Downstream(typ)
    states, logs, commit_vc = {}, {}, []
    for i, tx in enumerate(case["txns"]):
        x = tx["dc"]
        ss = po.vc_max([commit_vc[j] for j in tx.get("dep") or []])
        ss[x] = max(ss.get(x, 0), 10 * (i + 1) - 5)
        key = tx.get("key", "k")
        # the transaction's snapshot of the key: every earlier effect whose
        # commit VC is covered by ss (the materializer's own rule, done on dicts)
        st = po.crdt_new(typ)
        for _, p in reversed(logs.get(key, [])):
            oc = dict(p.snapshot_time)
            oc[p.commit_time[0]] = p.commit_time[1]
            if all(d in ss and t <= ss[d] for d, t in oc.items()):
                st = po.crdt_update(typ, p.op_param, st)
        for upd in tx["updates"]:
            eff = ds.effect(st, upd)
            st = po.crdt_update(typ, eff, st)
            lg = logs.setdefault(key, [])
            lg.insert(0, (len(lg) + 1, po.Payload(key, typ, eff, dict(ss), (x, 10 * (i + 1)),
                                                  i + 1)))
        cvc = dict(ss)
        cvc[x] = 10 * (i + 1)
        commit_vc.append(cvc)
    reads = []
    for r in case["reads"]:
        reads.append((r.get("key", "k"), po.vc_max([commit_vc[j] for j in r["at"]]), r["expect"]))
    return logs, reads
