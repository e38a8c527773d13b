"""Host mirror of stable_time_functions (src/stable_time_functions.erl) —
the GST merge plugin handed to meta_data_sender (src/antidote_sup.erl:100-103,
src/meta_data_sender.erl:112-115) — plus the cross-GPU exchange.

  export_funcs_and_vals() :39-40 -> [stable, UpdateFun, MergeFun, {}, {}]
  update_func_min(Last, Time) :42-48
  get_min_time(Dict) :51-85  — elementwise min on the device (agn_gst_min)
  update_stable(Last, New, UpdateFun) — meta_data_sender.erl:341-356 (agn_update_stable)

Clocks are dicts {dc: time}; a partition/node whose value is "undefined"
zeroes every DC of the result, as in the reference.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi
from ._lib import check, load

UNDEFINED = "undefined"


def update_func_min(last, time) -> bool:
    return True if last is None or last == UNDEFINED else time >= last


def export_funcs_and_vals():
    return ["stable", update_func_min, get_min_time, {}, {}]


def _engine(device):
    from .clocksi_materializer import engine
    return engine(device)


def encode_partitions(parts: dict):
    """{partition: dict | "undefined"} -> (dcs, clocks[P][D], defined[P])."""
    dcs = sorted({d for v in parts.values() if isinstance(v, dict) for d in v}, key=repr)
    index = {d: j for j, d in enumerate(dcs)}
    D, P = max(1, len(dcs)), len(parts)
    clocks = np.full((P, D), _abi.U64_MAX, np.uint64)
    defined = np.ones(P, np.uint8)
    for i, v in enumerate(parts.values()):
        if not isinstance(v, dict):
            defined[i] = 0
            continue
        for d, t in v.items():
            clocks[i, index[d]] = t
    return dcs, clocks, defined


def get_min_time(parts: dict, device: int = 0) -> dict:
    dcs, clocks, defined = encode_partitions(parts)
    if not parts:
        return {}
    D, P = clocks.shape[1], clocks.shape[0]
    eng = _engine(device)
    bc, bd, out = eng.upload(clocks), eng.upload(defined), eng.empty((D + 1) * 8)
    try:
        eng.gst_min(D, P, 1, bc.ptr, bd.ptr, out.ptr)
        eng.gst_finalize(D, 1, out.ptr)
        vec = eng.download(out, np.uint64, (D + 1,))
    finally:
        for b in (bc, bd, out):
            b.free()
    return {d: int(vec[j]) for j, d in enumerate(dcs) if int(vec[j]) != _abi.U64_MAX}


def update_stable(last_result: dict, new_dict: dict):
    """-> (Changed, NewResult) with update_func_min semantics."""
    dcs = sorted(set(last_result) | set(new_dict), key=repr)
    last = np.array([last_result.get(d, _abi.U64_MAX) for d in dcs] or [0], np.uint64)
    new = np.array([new_dict.get(d, _abi.U64_MAX) for d in dcs] or [0], np.uint64)
    ch = C.c_int(0)
    check(load().agn_update_stable(len(dcs), last.ctypes.data, new.ctypes.data, C.byref(ch)))
    return bool(ch.value), {d: int(last[j]) for j, d in enumerate(dcs)
                            if int(last[j]) != _abi.U64_MAX}


class GstExchange:
    """meta_data_sender's local-min -> all-nodes -> min round (:230-255) as one
    RCCL ncclMin allreduce of D+1 words: each rank reduces its own partitions
    on its GPU, the allreduce combines ranks (word D = "all defined"), then the
    undefined => 0 rule is applied once, after the exchange."""

    def __init__(self, dcs, nranks: int, rank: int, uid: bytes, device: int = 0):
        self.dcs = list(dcs)
        self.eng = _engine(device)
        if nranks > 1:
            self.eng.comm_init(nranks, rank, uid)
        self.nranks = nranks
        D = len(self.dcs)
        self.vec = self.eng.empty((D + 1) * 8)

    def epoch(self, local_parts: dict) -> dict:
        D = len(self.dcs)
        index = {d: j for j, d in enumerate(self.dcs)}
        P = len(local_parts)
        clocks = np.full((max(P, 1), D), _abi.U64_MAX, np.uint64)
        defined = np.ones(max(P, 1), np.uint8)
        for i, v in enumerate(local_parts.values()):
            if not isinstance(v, dict):
                defined[i] = 0
                continue
            for d, t in v.items():
                clocks[i, index[d]] = t
        bc, bd = self.eng.upload(clocks), self.eng.upload(defined)
        try:
            self.eng.gst_min(D, P, 1, bc.ptr, bd.ptr, self.vec.ptr)
            if self.nranks > 1:
                self.eng.gst_allreduce(self.vec.ptr, D + 1)
            self.eng.gst_finalize(D, 1, self.vec.ptr)
            vec = self.eng.download(self.vec, np.uint64, (D + 1,))
        finally:
            bc.free()
            bd.free()
        return {d: int(vec[j]) for j, d in enumerate(self.dcs) if int(vec[j]) != _abi.U64_MAX}
