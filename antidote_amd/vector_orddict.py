"""Host mirror of vector_orddict (src/vector_orddict.erl): the per-key
snapshot cache ordered newest first.  get_smaller/2 — the base-snapshot
selection on the read path (src/materializer_vnode.erl:400) — runs on the
device (agn_select_base); the batched form get_smaller_batch serves many
reads in one launch.  List surgery (insert, sublist, ...) is host-side."""
from __future__ import annotations

import numpy as np

from . import _abi
from .encode import DcTable, encode_clock, n_words


def _vc_get(vc, d):
    return vc.get(d, 0)


def _le(a, b):  # vectorclock:le, for host list maintenance (insert_bigger)
    return all(_vc_get(a, d) <= _vc_get(b, d) for d in set(a) | set(b))


def _all_dots_greater(a, b):
    return all(_vc_get(a, d) > _vc_get(b, d) for d in set(a) | set(b))


def _conc(a, b):
    return not _le(b, a) and not _le(a, b)


class VectorOrddict:
    def __init__(self, lst=None):
        self.lst = list(lst or [])

    @classmethod
    def new(cls):
        return cls()

    @classmethod
    def from_list(cls, lst):
        return cls(lst)

    def size(self):
        return len(self.lst)

    def to_list(self):
        return list(self.lst)

    def first(self):
        return self.lst[0]

    def last(self):
        return self.lst[-1]

    def get_smaller(self, vector, device: int = 0):
        """-> ((Clock, Val) | None, IsFirst)"""
        return get_smaller_batch([(vector, self)], device)[0]

    def get_smaller_from_id(self, dc, time):
        for clock, val in self.lst:
            if _vc_get(clock, dc) <= time:
                return clock, val
        return None

    def insert(self, vector, val):
        for i, (clock, _) in enumerate(self.lst):
            if _all_dots_greater(vector, clock):
                return VectorOrddict(self.lst[:i] + [(vector, val)] + self.lst[i:])
        return VectorOrddict(self.lst + [(vector, val)])

    def insert_bigger(self, vector, val):
        if not self.lst:
            return VectorOrddict([(vector, val)])
        if not _le(vector, self.lst[0][0]):
            return VectorOrddict([(vector, val)] + self.lst)
        return VectorOrddict(self.lst)

    def sublist(self, start, length):
        return VectorOrddict(self.lst[start - 1:start - 1 + length])

    def filter(self, fun):
        return VectorOrddict([x for x in self.lst if fun(x)])

    def is_concurrent_with_any(self, other):
        return any(_conc(c, other) for c, _ in self.lst)


def get_smaller_batch(items, device: int = 0):
    """[(ReadClock, VectorOrddict)] -> [((Clock, Val) | None, IsFirst)], one launch."""
    from .clocksi_materializer import engine
    if not items:
        return []
    dcs = DcTable()
    for r, d in items:
        for dc in r:
            dcs.id(dc)
        for c, _ in d.lst:
            for dc in c:
                dcs.id(dc)
    D = max(1, len(dcs))
    W = n_words(D)
    n = len(items)
    off = np.zeros(n + 1, np.uint64)
    for i, (_, d) in enumerate(items):
        off[i + 1] = off[i] + d.size()
    M = max(int(off[-1]), 1)
    clocks = np.zeros((M, D), np.uint64)
    cmask = np.zeros((M, W), np.uint64)
    R = np.zeros((n, D), np.uint64)
    Rm = np.zeros((n, W), np.uint64)
    j = 0
    for i, (r, d) in enumerate(items):
        R[i], Rm[i] = encode_clock(r, dcs, D)
        for c, _ in d.lst:
            clocks[j], cmask[j] = encode_clock(c, dcs, D)
            j += 1
    eng = engine(device)
    bufs = [eng.upload(x) for x in (off, clocks, cmask, R, Rm)]
    oi, of = eng.empty(n * 4), eng.empty(n)
    try:
        eng.select_base(D, n, *[b.ptr for b in bufs], oi.ptr, of.ptr)
        idx = eng.download(oi, np.int32, (n,))
        first = eng.download(of, np.uint8, (n,))
    finally:
        for b in bufs + [oi, of]:
            b.free()
    out = []
    for i, (_, d) in enumerate(items):
        k = int(idx[i])
        out.append((None if k < 0 else d.lst[k], bool(first[i])))
    return out


__all__ = ["VectorOrddict", "get_smaller_batch", "_abi"]
