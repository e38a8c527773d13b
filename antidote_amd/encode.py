"""Host-side encoding of Erlang-shaped materializer inputs into the SoA layout.

This is the work the NIF (nif/antidote_gpu_nif.c) does when a term crosses
the boundary: DC ids (arbitrary terms, include/antidote.hrl:187) are mapped
to column indices, vector clocks (dicts, :188) become dense rows plus a
presence bitmask, #clocksi_payload{} records (:197-204) become SoA entries
with OpSSCommit precomputed (src/clocksi_materializer.erl:224), and CRDT
effects / set elements / register values / tokens are interned to integers.

Pure numpy: usable without a GPU (the CPU tests exercise it directly).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Iterable

import numpy as np

from . import _abi

IGNORE = "ignore"


@dataclass
class ClocksiPayload:
    """#clocksi_payload{key, type, op_param, snapshot_time, commit_time, txid}."""
    key: Any
    type: str
    op_param: Any
    snapshot_time: dict
    commit_time: tuple
    txid: Any = None


class Interner:
    """Term -> dense integer id (ids start at `first`)."""

    def __init__(self, first: int = 0):
        self._ids: dict = {}
        self._terms: list = []
        self._first = first

    @staticmethod
    def _key(term):
        return (type(term).__name__, repr(term))

    def id(self, term) -> int:
        k = self._key(term)
        i = self._ids.get(k)
        if i is None:
            i = self._first + len(self._terms)
            self._ids[k] = i
            self._terms.append(term)
        return i

    def term(self, i: int):
        return self._terms[i - self._first]

    def __len__(self):
        return len(self._terms)


class DcTable(Interner):
    """dcid() -> column index."""


def n_words(n_dcs: int) -> int:
    return (n_dcs + 63) // 64


def encode_clock(vc: dict, dcs: DcTable, n_dcs: int):
    """dict clock -> (values[D] u64, mask[W] u64)."""
    vals = np.zeros(n_dcs, np.uint64)
    mask = np.zeros(n_words(n_dcs), np.uint64)
    for dc, t in vc.items():
        d = dcs.id(dc)
        if d >= n_dcs:
            raise ValueError(f"DC table overflow: {dc!r} needs more than {n_dcs} columns")
        if not (0 <= int(t) < _abi.U64_MAX):
            raise ValueError(f"clock value out of range: {t!r}")
        vals[d] = int(t)
        mask[d >> 6] |= np.uint64(1 << (d & 63))
    return vals, mask


def decode_clock(vals, mask, dcs: DcTable) -> dict:
    out = {}
    for d in range(len(vals)):
        if (int(mask[d >> 6]) >> (d & 63)) & 1:
            out[dcs.term(d)] = int(vals[d])
    return out


def op_ss_commit(p: ClocksiPayload) -> dict:
    """OpSSCommit = dict:store(OpDc, OpCommitTime, OperationSnapshotTime)."""
    dc, t = p.commit_time
    oc = dict(p.snapshot_time)
    oc[dc] = t
    return oc


@dataclass
class EncodedLog:
    """numpy arrays for one agn_log (host side)."""
    crdt_type: int
    n_dcs: int
    key_off: np.ndarray
    key_type: np.ndarray
    oc: np.ndarray
    oc_mask: np.ndarray | None
    op_id: np.ndarray
    txid: np.ndarray
    eff: np.ndarray | None = None
    tag: np.ndarray | None = None
    add_tok: np.ndarray | None = None
    rem_off: np.ndarray | None = None
    rem_tok: np.ndarray | None = None
    invalid_terms: dict = field(default_factory=dict)  # entry -> original effect term
    entry_op: list = field(default_factory=list)       # entry -> (key index, op position)

    @property
    def n_keys(self):
        return len(self.key_off) - 1

    @property
    def n_entries(self):
        return int(self.key_off[-1])


class LogEncoder:
    """Builds the SoA log key by key; ops are given OLDEST first, each as
    (op_id, ClocksiPayload) — the order of the ETS ops tuple."""

    def __init__(self, crdt_type: int, n_dcs: int, dcs: DcTable | None = None,
                 dense: bool = False, tags: Interner | None = None,
                 tokens: Interner | None = None, txids: Interner | None = None):
        self.crdt_type = crdt_type
        self.n_dcs = n_dcs
        self.W = n_words(n_dcs)
        self.dcs = dcs or DcTable()
        self.dense = dense
        self.tags = tags or Interner(0)
        self.tokens = tokens or Interner(1)
        self.txids = txids or Interner(1)
        self._key_off = [0]
        self._key_type = []
        self._oc, self._ocm, self._id, self._tx = [], [], [], []
        self._eff, self._tag, self._add, self._rem_off, self._rem = [], [], [], [0], []
        self._invalid = {}
        self._entry_op = []

    def _entries_for(self, effect):
        """Split one effect into (tag, add_tok, [rem_toks]) entries, or None if
        the effect cannot be represented (-> invalid entry)."""
        t = self.crdt_type
        try:
            if t == _abi.SET_AW:
                ents = []
                for elem, adds, rems in effect:
                    adds, rems = list(adds), list(rems)
                    rem_ids = [self.tokens.id(x) for x in rems]
                    if not adds:
                        ents.append((self.tags.id(elem), 0, rem_ids))
                    for j, a in enumerate(adds):
                        ents.append((self.tags.id(elem), self.tokens.id(a),
                                     rem_ids if j == 0 else []))
                return ents
            if t == _abi.REGISTER_MV:
                if isinstance(effect, tuple) and len(effect) == 2 and effect[0] == "reset":
                    return [(0, 0, [self.tokens.id(x) for x in effect[1]])]
                value, token, ovr = effect
                return [(self.tags.id(value), self.tokens.id(token),
                         [self.tokens.id(x) for x in ovr])]
        except (TypeError, ValueError):
            return None
        return None

    def add_key(self, ops: Iterable, key_type: int | None = None) -> int:
        k = len(self._key_off) - 1
        types = set()
        pos = 0
        for op_id, p in ops:
            types.add(p.type)
            oc = op_ss_commit(p)
            vals, mask = encode_clock(oc, self.dcs, self.n_dcs)
            txid = 0 if p.txid is None else self.txids.id(p.txid)
            if self.crdt_type == _abi.COUNTER_PN:
                e = p.op_param
                ok = isinstance(e, int) and not isinstance(e, bool) and \
                    -(1 << 63) < e < (1 << 63)
                ents = [(e if ok else _abi.EFFECT_INVALID, None, None)]
                if not ok:
                    self._invalid[len(self._id)] = e
            else:
                ents = self._entries_for(p.op_param)
                if ents is None:
                    self._invalid[len(self._id)] = p.op_param
                    ents = [(_abi.TAG_INVALID, 0, [])]
            for tag, add, rems in ents:
                self._oc.append(vals)
                self._ocm.append(mask)
                self._id.append(op_id)
                self._tx.append(txid)
                self._entry_op.append((k, pos))
                if self.crdt_type == _abi.COUNTER_PN:
                    self._eff.append(tag)
                else:
                    self._tag.append(tag)
                    self._add.append(add)
                    self._rem.extend(rems)
                    self._rem_off.append(len(self._rem))
            pos += 1
        self._key_off.append(len(self._id))
        if key_type is None:
            if not types:
                key_type = self.crdt_type
            elif len(types) == 1:
                key_type = _abi.TYPE_IDS.get(next(iter(types)), 0xFE)
            else:
                key_type = _abi.TYPE_MIXED
        self._key_type.append(key_type)
        return k

    def build(self) -> EncodedLog:
        D, W = self.n_dcs, self.W
        n = len(self._id)
        oc = np.array(self._oc, np.uint64).reshape(n, D) if n else np.zeros((0, D), np.uint64)
        ocm = np.array(self._ocm, np.uint64).reshape(n, W) if n else np.zeros((0, W), np.uint64)
        full = np.uint64(_abi.U64_MAX)
        if self.dense:
            want = np.zeros(W, np.uint64)
            for d in range(D):
                want[d >> 6] |= np.uint64(1 << (d & 63))
            if n and not (ocm == want).all():
                raise ValueError("dense log requested but an op clock is sparse")
            ocm = None
        del full
        log = EncodedLog(
            crdt_type=self.crdt_type, n_dcs=D,
            key_off=np.array(self._key_off, np.uint64),
            key_type=np.array(self._key_type, np.uint8),
            oc=oc, oc_mask=ocm, op_id=np.array(self._id, np.uint32),
            txid=np.array(self._tx, np.uint64), invalid_terms=self._invalid,
            entry_op=self._entry_op)
        if self.crdt_type == _abi.COUNTER_PN:
            log.eff = np.array(self._eff, np.int64)
        else:
            log.tag = np.array(self._tag, np.uint32)
            log.add_tok = np.array(self._add, np.uint64)
            log.rem_off = np.array(self._rem_off, np.uint32)
            log.rem_tok = np.array(self._rem, np.uint64)
        return log


@dataclass
class EncodedRead:
    n_dcs: int
    req_type: int
    keys: np.ndarray
    R: np.ndarray
    R_mask: np.ndarray
    sct: np.ndarray
    sct_mask: np.ndarray
    sct_ignore: np.ndarray
    txid: np.ndarray
    base_value: np.ndarray
    base_off: np.ndarray
    base_tag: np.ndarray
    base_tok: np.ndarray

    @property
    def n_req(self):
        return len(self.keys)


class ReadEncoder:
    """One materialize/4 request per key: (key index, MinSnapshotTime, SCT or
    ignore, TxId or ignore, base value)."""

    def __init__(self, enc: LogEncoder, req_type: int | None = None):
        self.enc = enc
        self.req_type = enc.crdt_type if req_type is None else req_type
        self.rows = []

    def add(self, key: int, R: dict, sct=IGNORE, txid=IGNORE, base=None):
        self.rows.append((key, R, sct, txid, base))

    def build(self) -> EncodedRead:
        e = self.enc
        D, W = e.n_dcs, e.W
        n = len(self.rows)
        R = np.zeros((n, D), np.uint64)
        Rm = np.zeros((n, W), np.uint64)
        S = np.zeros((n, D), np.uint64)
        Sm = np.zeros((n, W), np.uint64)
        Si = np.zeros(n, np.uint8)
        T = np.zeros(n, np.uint64)
        BV = np.zeros(n, np.int64)
        boff, btag, btok = [0], [], []
        for i, (key, r, sct, txid, base) in enumerate(self.rows):
            R[i], Rm[i] = encode_clock(r, e.dcs, D)
            if sct == IGNORE or sct is None:
                Si[i] = 1
            else:
                S[i], Sm[i] = encode_clock(sct, e.dcs, D)
            if txid not in (IGNORE, None):
                T[i] = e.txids.id(txid)
            if e.crdt_type == _abi.COUNTER_PN:
                BV[i] = 0 if base is None else int(base)
            else:
                for tag_term, toks in (base or []):
                    for tk in (toks if e.crdt_type == _abi.SET_AW else [toks]):
                        btag.append(e.tags.id(tag_term))
                        btok.append(e.tokens.id(tk))
            boff.append(len(btag))
        return EncodedRead(D, self.req_type, np.array([r[0] for r in self.rows], np.uint64),
                           R, Rm, S, Sm, Si, T, BV, np.array(boff, np.uint64),
                           np.array(btag, np.uint32), np.array(btok, np.uint64))


def state_capacity(log: EncodedLog, req: EncodedRead) -> np.ndarray:
    """Upper bound of live pairs per request (adding entries + base pairs)."""
    adds = (log.add_tok != 0).astype(np.uint64) if log.add_tok is not None else None
    cap = np.zeros(req.n_req + 1, np.uint64)
    for i, k in enumerate(req.keys):
        a, b = int(log.key_off[k]), int(log.key_off[k + 1])
        c = int(adds[a:b].sum()) if adds is not None else 0
        c += int(req.base_off[i + 1] - req.base_off[i])
        cap[i + 1] = cap[i] + c
    return cap


# ---------------------------------------------------------------- ctypes views
def ptr(a) -> int | None:
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        if a.size == 0:
            return None
        assert a.flags["C_CONTIGUOUS"]
        return a.ctypes.data
    return int(a)  # already a device address


def log_struct(log, dense_mask: bool = True) -> _abi.AgnLog:
    s = _abi.AgnLog()
    s.crdt_type, s.n_dcs = log.crdt_type, log.n_dcs
    s.n_keys, s.n_entries = log.n_keys, log.n_entries
    s.key_off, s.key_type = ptr(log.key_off), ptr(log.key_type)
    s.oc, s.oc_mask, s.op_id, s.txid = ptr(log.oc), ptr(log.oc_mask), ptr(log.op_id), ptr(log.txid)
    s.eff, s.tag, s.add_tok = ptr(log.eff), ptr(log.tag), ptr(log.add_tok)
    s.rem_off, s.rem_tok = ptr(log.rem_off), ptr(log.rem_tok)
    if log.rem_off is not None and s.rem_off is None:
        raise ValueError("rem_off must have n_entries+1 elements")
    return s


def read_struct(req: EncodedRead, sparse: bool = True) -> _abi.AgnRead:
    s = _abi.AgnRead()
    s.n_req = req.n_req
    s.keys = ptr(req.keys)
    s.R, s.R_mask = ptr(req.R), ptr(req.R_mask) if sparse else None
    s.sct, s.sct_mask = ptr(req.sct), ptr(req.sct_mask) if sparse else None
    s.sct_ignore, s.txid = ptr(req.sct_ignore), ptr(req.txid)
    s.req_type = req.req_type
    s.base_value, s.base_off = ptr(req.base_value), ptr(req.base_off)
    s.base_tag, s.base_tok = ptr(req.base_tag), ptr(req.base_tok)
    return s


@dataclass
class ResultArrays:
    value: np.ndarray
    hole: np.ndarray
    lastct: np.ndarray
    lastct_mask: np.ndarray | None
    count: np.ndarray
    flags: np.ndarray
    err_pos: np.ndarray
    out_off: np.ndarray | None = None
    out_n: np.ndarray | None = None
    out_tag: np.ndarray | None = None
    out_tok: np.ndarray | None = None


def alloc_result(n_req: int, n_dcs: int, sparse: bool, cap_off=None) -> ResultArrays:
    W = n_words(n_dcs)
    r = ResultArrays(
        value=np.zeros(n_req, np.int64), hole=np.zeros(n_req, np.int64),
        lastct=np.zeros((n_req, n_dcs), np.uint64),
        lastct_mask=np.zeros((n_req, W), np.uint64) if sparse else None,
        count=np.zeros(n_req, np.uint32), flags=np.zeros(n_req, np.uint32),
        err_pos=np.zeros(n_req, np.uint32))
    if cap_off is not None:
        total = int(cap_off[-1])
        r.out_off = np.ascontiguousarray(cap_off, np.uint64)
        r.out_n = np.zeros(n_req, np.uint32)
        r.out_tag = np.zeros(max(total, 1), np.uint32)
        r.out_tok = np.zeros(max(total, 1), np.uint64)
    return r


def result_struct(r: ResultArrays) -> _abi.AgnResult:
    s = _abi.AgnResult()
    s.value, s.hole, s.lastct, s.lastct_mask = ptr(r.value), ptr(r.hole), ptr(r.lastct), ptr(r.lastct_mask)
    s.count, s.flags, s.err_pos = ptr(r.count), ptr(r.flags), ptr(r.err_pos)
    s.out_off, s.out_n = ptr(r.out_off), ptr(r.out_n)
    s.out_tag, s.out_tok = ptr(r.out_tag), ptr(r.out_tok)
    return s
