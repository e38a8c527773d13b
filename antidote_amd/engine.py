"""Thin object wrapper over the C ABI: a device context, device buffers,
device-resident op logs / read batches / results, and the batched entry
points.  Everything numeric happens in libantidote_gpu.so."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _abi
from ._lib import EngineUnavailable, check, load
from .encode import (EncodedLog, EncodedRead, ResultArrays, alloc_result, log_struct, n_words,
                     read_struct, result_struct)


class DevBuf:
    """HBM allocation owned by an Engine (agn_dev_alloc)."""

    def __init__(self, eng: "Engine", nbytes: int):
        self.eng, self.nbytes = eng, int(nbytes)
        p = C.c_void_p()
        check(eng.lib.agn_dev_alloc(eng.ctx, self.nbytes, C.byref(p)), "agn_dev_alloc")
        self.ptr = p.value or 0
        eng._bufs.add(self)

    def free(self):
        if self.ptr:
            self.eng.lib.agn_dev_free(self.eng.ctx, self.ptr)
            self.ptr = 0
        self.eng._bufs.discard(self)


@dataclass
class DeviceArrays:
    """Device copies of an Encoded* / Result structure (same field names)."""
    struct: object
    bufs: dict = field(default_factory=dict)
    shapes: dict = field(default_factory=dict)


class Engine:
    def __init__(self, device: int = 0):
        self.lib = load()
        self.ctx = C.c_void_p()
        rc = self.lib.agn_open(device, C.byref(self.ctx))
        if rc in (_abi.ENODEV, _abi.ENOTSUP):
            raise EngineUnavailable(self.lib.agn_last_error().decode())
        check(rc, "agn_open")
        self.device = device
        self._bufs: set = set()

    # ---------------------------------------------------------------- memory
    def close(self):
        for b in list(self._bufs):
            b.free()
        if self.ctx:
            self.lib.agn_close(self.ctx)
            self.ctx = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def upload(self, arr: np.ndarray | None) -> DevBuf | None:
        if arr is None:
            return None
        arr = np.ascontiguousarray(arr)
        b = DevBuf(self, max(arr.nbytes, 8))
        if arr.nbytes:
            check(self.lib.agn_memcpy_h2d(self.ctx, b.ptr, arr.ctypes.data, arr.nbytes, None))
        return b

    def empty(self, nbytes: int) -> DevBuf:
        return DevBuf(self, max(int(nbytes), 8))

    def download(self, buf: DevBuf, dtype, shape, stream=None) -> np.ndarray:
        out = np.empty(shape, dtype)
        if out.nbytes:
            check(self.lib.agn_memcpy_d2h(self.ctx, out.ctypes.data, buf.ptr, out.nbytes, stream))
            check(self.lib.agn_stream_sync(self.ctx, stream))
        return out

    def sync(self, stream=None):
        check(self.lib.agn_stream_sync(self.ctx, stream))

    # ---------------------------------------------------------------- materialize
    def materialize_host(self, log: EncodedLog, req: EncodedRead, sparse: bool = True,
                         cap_off=None) -> ResultArrays:
        """Host arrays in, host arrays out (agn_materialize_host)."""
        res = alloc_result(req.n_req, log.n_dcs, sparse=sparse, cap_off=cap_off)
        ls, rs, os_ = log_struct(log), read_struct(req, sparse=sparse), result_struct(res)
        if not sparse:
            ls.oc_mask = None
        check(self.lib.agn_materialize_host(self.ctx, C.byref(ls), C.byref(rs), C.byref(os_)),
              "agn_materialize_host")
        return res

    def upload_log(self, log: EncodedLog) -> DeviceArrays:
        s = log_struct(log)
        d = DeviceArrays(s)
        for name in ("key_off", "key_type", "oc", "oc_mask", "op_id", "txid", "eff", "tag",
                     "add_tok", "rem_off", "rem_tok"):
            a = getattr(log, name)
            if a is None or (isinstance(a, np.ndarray) and a.size == 0 and name != "rem_tok"):
                setattr(s, name, None)
                continue
            b = self.upload(a)
            d.bufs[name] = b
            setattr(s, name, b.ptr)
        return d

    def index_ids(self, dlog, stream=None) -> DevBuf:
        """Build agn_log.key_id0 (consecutive op-id base per key, agn_log_index_ids)
        for a device log and attach it; returns the buffer (owned by dlog when
        dlog is DeviceArrays)."""
        ls = dlog.struct if isinstance(dlog, DeviceArrays) else dlog
        b = self.empty(max(1, int(ls.n_keys)) * 4)
        check(self.lib.agn_log_index_ids(self.ctx, C.byref(ls), b.ptr, stream),
              "agn_log_index_ids")
        ls.key_id0 = b.ptr
        if isinstance(dlog, DeviceArrays):
            dlog.bufs["key_id0"] = b
        return b

    def index_masks(self, dlog, stream=None) -> DevBuf:
        """Build agn_log.key_mask (the DC set every entry of a key carries, 0
        when they differ; agn_log_index_masks) for a device log and attach it."""
        ls = dlog.struct if isinstance(dlog, DeviceArrays) else dlog
        b = self.empty(max(1, int(ls.n_keys)) * 8)
        check(self.lib.agn_log_index_masks(self.ctx, C.byref(ls), b.ptr, stream),
              "agn_log_index_masks")
        ls.key_mask = b.ptr
        if isinstance(dlog, DeviceArrays):
            dlog.bufs["key_mask"] = b
        return b

    def alloc_log_like(self, log: EncodedLog) -> DeviceArrays:
        """Device arrays with the sizes (and presence) of `log`'s (agn_prune_ops output)."""
        s = _abi.AgnLog()
        s.crdt_type, s.n_dcs = log.crdt_type, log.n_dcs
        s.n_keys, s.n_entries = log.n_keys, log.n_entries
        d = DeviceArrays(s)
        for name in ("key_off", "oc", "oc_mask", "op_id", "txid", "eff", "tag", "add_tok",
                     "rem_off", "rem_tok"):
            a = getattr(log, name)
            if a is None or (isinstance(a, np.ndarray) and a.size == 0 and name != "rem_tok"):
                setattr(s, name, None)
                continue
            b = self.empty(a.nbytes)
            d.bufs[name] = b
            d.shapes[name] = (a.dtype, a.shape)
            setattr(s, name, b.ptr)
        return d

    def ss_lookup(self, cache, n_req, keys_ptr, R_ptr, Rm_ptr, sct_ptr, sctm_ptr, ign_ptr,
                  base_ptr, first_ptr, status_ptr, stream=None):
        check(self.lib.agn_ss_lookup(self.ctx, C.byref(cache), n_req, keys_ptr, R_ptr, Rm_ptr,
                                     sct_ptr, sctm_ptr, ign_ptr, base_ptr, first_ptr, status_ptr,
                                     stream), "agn_ss_lookup")

    def ss_store(self, cache, dlog, n_req, keys_ptr, first_ptr, status_ptr, gc_ptr, dres,
                 handle_ptr, prune_ptr, thr_ptr, thrm_ptr, stream=None):
        ls = dlog.struct if isinstance(dlog, DeviceArrays) else dlog
        rs = dres.struct if isinstance(dres, DeviceArrays) else dres
        check(self.lib.agn_ss_store(self.ctx, C.byref(cache), C.byref(ls), n_req, keys_ptr,
                                    first_ptr, status_ptr, gc_ptr, C.byref(rs), handle_ptr,
                                    prune_ptr, thr_ptr, thrm_ptr, stream), "agn_ss_store")

    def read_cached(self, cache, dlog, n_req, keys_ptr, R_ptr, txid_ptr, gc_ptr, dres,
                    status_ptr, prune_ptr, thr_ptr, stream=None):
        """agn_read_cached: read/6 for a batch in one kernel (ss_lookup ->
        materialize -> ss_store), counter_pn with dense clocks, D <= 8."""
        ls = dlog.struct if isinstance(dlog, DeviceArrays) else dlog
        rs = dres.struct if isinstance(dres, DeviceArrays) else dres
        check(self.lib.agn_read_cached(self.ctx, C.byref(cache), C.byref(ls), n_req, keys_ptr,
                                       R_ptr, txid_ptr, gc_ptr, C.byref(rs), status_ptr,
                                       prune_ptr, thr_ptr, stream), "agn_read_cached")

    def prune_ops(self, dlog: DeviceArrays, prune_ptr, thr_ptr, thr_mask_ptr, dout: DeviceArrays,
                  flags_ptr=None, totals_ptr=None, stream=None):
        """agn_prune_ops: materializer_vnode GC of the device op log (out of place)."""
        check(self.lib.agn_prune_ops(self.ctx, C.byref(dlog.struct), prune_ptr, thr_ptr,
                                     thr_mask_ptr, C.byref(dout.struct), flags_ptr, totals_ptr,
                                     stream), "agn_prune_ops")

    def upload_read(self, req: EncodedRead, sparse: bool = True) -> DeviceArrays:
        s = read_struct(req, sparse=sparse)
        d = DeviceArrays(s)
        names = ["keys", "R", "sct", "sct_ignore", "txid", "base_value", "base_off", "base_tag",
                 "base_tok"] + (["R_mask", "sct_mask"] if sparse else [])
        for name in names:
            if getattr(s, name) is None:
                continue
            b = self.upload(getattr(req, name))
            d.bufs[name] = b
            setattr(s, name, b.ptr)
        return d

    def alloc_result(self, n_req: int, n_dcs: int, sparse: bool, cap_off=None) -> DeviceArrays:
        s = _abi.AgnResult()
        d = DeviceArrays(s)
        W = n_words(n_dcs)
        spec = {"value": (np.int64, (n_req,)), "hole": (np.int64, (n_req,)),
                "lastct": (np.uint64, (n_req, n_dcs)), "count": (np.uint32, (n_req,)),
                "flags": (np.uint32, (n_req,)), "err_pos": (np.uint32, (n_req,))}
        if sparse:
            spec["lastct_mask"] = (np.uint64, (n_req, W))
        if cap_off is not None:
            total = max(int(cap_off[-1]), 1)
            spec.update({"out_n": (np.uint32, (n_req,)), "out_tag": (np.uint32, (total,)),
                         "out_tok": (np.uint64, (total,))})
            b = self.upload(np.ascontiguousarray(cap_off, np.uint64))
            d.bufs["out_off"] = b
            d.shapes["out_off"] = (np.uint64, (n_req + 1,))
            s.out_off = b.ptr
        for name, (dt, shape) in spec.items():
            b = self.empty(int(np.prod(shape)) * np.dtype(dt).itemsize)
            d.bufs[name] = b
            d.shapes[name] = (dt, shape)
            setattr(s, name, b.ptr)
        return d

    def fetch_result(self, d: DeviceArrays, stream=None) -> ResultArrays:
        """The results in host arrays; a request flagged AGN_F_CT_FULL (a
        batch with AGN_HINT_CT_FLAG) gets its LastOpCt mask back -- every
        column -- and the flag is cleared, so results compare as without the
        hint."""
        get = {n: self.download(d.bufs[n], *d.shapes[n], stream=stream) for n in d.shapes}
        full = (get["flags"] & _abi.F_CT_FULL) != 0
        if full.any():
            D = get["lastct"].shape[1]
            if get.get("lastct_mask") is not None:
                row = np.zeros(get["lastct_mask"].shape[1], np.uint64)
                for w in range(row.size):
                    bits = min(64, D - 64 * w)
                    row[w] = np.uint64((1 << bits) - 1) if bits > 0 else np.uint64(0)
                get["lastct_mask"][full] = row
            get["flags"] &= np.uint32(~_abi.F_CT_FULL & 0xFFFFFFFF)
        return ResultArrays(value=get["value"], hole=get["hole"], lastct=get["lastct"],
                            lastct_mask=get.get("lastct_mask"), count=get["count"],
                            flags=get["flags"], err_pos=get["err_pos"], out_off=get.get("out_off"),
                            out_n=get.get("out_n"), out_tag=get.get("out_tag"),
                            out_tok=get.get("out_tok"))

    def materialize(self, dlog, dreq, dres, stream=None):
        ls = dlog.struct if isinstance(dlog, DeviceArrays) else dlog
        rs = dreq.struct if isinstance(dreq, DeviceArrays) else dreq
        os_ = dres.struct if isinstance(dres, DeviceArrays) else dres
        check(self.lib.agn_materialize(self.ctx, C.byref(ls), C.byref(rs), C.byref(os_), stream),
              "agn_materialize")

    def bind_materialize(self, dlog, dreq, dres, stream=None):
        """agn_materialize with its arguments converted once: returns a
        zero-argument callable for repeated launches of the same batch (a
        small batch's step is otherwise dominated by the per-call ctypes
        argument conversion)."""
        ls = dlog.struct if isinstance(dlog, DeviceArrays) else dlog
        rs = dreq.struct if isinstance(dreq, DeviceArrays) else dreq
        os_ = dres.struct if isinstance(dres, DeviceArrays) else dres
        fn, ctx = self.lib.agn_materialize, self.ctx
        args = (ctx, C.byref(ls), C.byref(rs), C.byref(os_), stream)
        keep = (ls, rs, os_)  # the structs outlive the callable

        def call(_fn=fn, _args=args, _keep=keep):
            rc = _fn(*_args)
            if rc:
                check(rc, "agn_materialize")
        return call

    def tune(self, dlog, dreq, dres, stream=None, rounds=3):
        """agn_tune: time the bit-identical kernel variants of this batch's
        path, select the fastest for this device; returns (choice, ms) with
        choice -1 (nothing to tune), 0 (VGPR rows), 1 (LDS-DMA rows) or 2
        (quad rows, D = 8) and ms = fastest launch per variant (0 where the
        shape lacks it).  Blocks; dres holds the results."""
        ls = dlog.struct if isinstance(dlog, DeviceArrays) else dlog
        rs = dreq.struct if isinstance(dreq, DeviceArrays) else dreq
        os_ = dres.struct if isinstance(dres, DeviceArrays) else dres
        choice = C.c_int(-1)
        ms = (C.c_float * 3)()
        check(self.lib.agn_tune(self.ctx, C.byref(ls), C.byref(rs), C.byref(os_), stream,
                                int(rounds), C.byref(choice), ms), "agn_tune")
        return choice.value, (ms[0], ms[1], ms[2])

    # ---------------------------------------------------------------- generator
    def gen_dev(self, cfg: _abi.AgnGenCfg, stream=None):
        log, req = _abi.AgnLog(), _abi.AgnRead()
        check(self.lib.agn_gen_dev(self.ctx, C.byref(cfg), C.byref(log), C.byref(req), stream),
              "agn_gen_dev")
        return log, req

    def free_gen(self, log, req):
        check(self.lib.agn_gen_free_dev(self.ctx, C.byref(log), C.byref(req)))

    # ---------------------------------------------------------------- GST
    def gst_min(self, n_dcs, n_parts, n_epochs, clocks_ptr, defined_ptr, out_ptr, stream=None):
        check(self.lib.agn_gst_min(self.ctx, n_dcs, n_parts, n_epochs, clocks_ptr, defined_ptr,
                                   out_ptr, stream), "agn_gst_min")

    def gst_finalize(self, n_dcs, n_epochs, vec_ptr, stream=None):
        check(self.lib.agn_gst_finalize(self.ctx, n_dcs, n_epochs, vec_ptr, stream),
              "agn_gst_finalize")

    def gst_scalar(self, n_dcs, n_epochs, vec_ptr, out_ptr, stream=None):
        check(self.lib.agn_gst_scalar(self.ctx, n_dcs, n_epochs, vec_ptr, out_ptr, stream),
              "agn_gst_scalar")

    def dep_check(self, n_dcs, n_txn, deps_ptr, dmask_ptr, origin_ptr, part_ptr, n_parts,
                  pc_ptr, pmask_ptr, out_ptr, stream=None):
        check(self.lib.agn_dep_check(self.ctx, n_dcs, n_txn, deps_ptr, dmask_ptr, origin_ptr,
                                     part_ptr, n_parts, pc_ptr, pmask_ptr, out_ptr, stream),
              "agn_dep_check")

    def select_base(self, n_dcs, n_req, off_ptr, clocks_ptr, cmask_ptr, R_ptr, Rmask_ptr,
                    idx_ptr, first_ptr, stream=None):
        check(self.lib.agn_select_base(self.ctx, n_dcs, n_req, off_ptr, clocks_ptr, cmask_ptr,
                                       R_ptr, Rmask_ptr, idx_ptr, first_ptr, stream),
              "agn_select_base")

    # ---------------------------------------------------------------- RCCL
    @staticmethod
    def unique_id() -> bytes:
        lib = load()
        buf = (C.c_uint8 * _abi.UNIQUE_ID_BYTES)()
        check(lib.agn_comm_unique_id(buf), "agn_comm_unique_id")
        return bytes(buf)

    def comm_init(self, nranks: int, rank: int, uid: bytes):
        buf = (C.c_uint8 * _abi.UNIQUE_ID_BYTES).from_buffer_copy(uid)
        check(self.lib.agn_comm_init(self.ctx, nranks, rank, buf), "agn_comm_init")

    def gst_allreduce(self, vec_ptr, n_words_, stream=None):
        check(self.lib.agn_gst_allreduce(self.ctx, vec_ptr, n_words_, stream), "agn_gst_allreduce")


def _ptr(a):
    return None if a is None else a.ctypes.data


class OpLog:
    """Engine-owned per-partition op log (agn_oplog_*): the materializer_vnode
    ETS ops cache (src/materializer_vnode.erl:621-647) resident in HBM.
    `append` mirrors op_insert_gc for a batch of entries (host arrays),
    `flush` returns the device view (an AgnLog with key_len) for
    Engine.materialize / ss_store, `prune` is snapshot_insert_gc's
    prune_ops + ETS resize."""

    def __init__(self, eng: Engine, crdt_type: int, n_dcs: int, n_keys: int,
                 sparse: bool = False, init_slots: int = 0):
        self.eng, self.crdt_type, self.n_dcs, self.n_keys = eng, crdt_type, n_dcs, n_keys
        self.sparse = sparse
        self.h = C.c_void_p()
        check(eng.lib.agn_oplog_create(eng.ctx, crdt_type, n_dcs, n_keys, int(sparse),
                                       init_slots, C.byref(self.h)), "agn_oplog_create")

    def close(self):
        if self.h:
            self.eng.lib.agn_oplog_destroy(self.h)
            self.h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def append(self, keys, oc, *, oc_mask=None, txid=None, eff=None, tag=None, add_tok=None,
               rem_off=None, rem_tok=None, same_op=None):
        """Returns (op_id[n] u32, gc_due[n] u8)."""
        keys = np.ascontiguousarray(keys, np.uint64)
        n = len(keys)
        cv = lambda a, dt: None if a is None else np.ascontiguousarray(a, dt)  # noqa: E731
        oc, oc_mask, txid = cv(oc, np.uint64), cv(oc_mask, np.uint64), cv(txid, np.uint64)
        eff, tag, add_tok = cv(eff, np.int64), cv(tag, np.uint32), cv(add_tok, np.uint64)
        rem_off, rem_tok, same_op = cv(rem_off, np.uint32), cv(rem_tok, np.uint64), \
            cv(same_op, np.uint8)
        if rem_tok is not None and rem_tok.size == 0:
            rem_tok = np.zeros(1, np.uint64)
        ids, due = np.zeros(n, np.uint32), np.zeros(n, np.uint8)
        check(self.eng.lib.agn_oplog_append(
            self.h, n, _ptr(keys), _ptr(same_op), _ptr(oc), _ptr(oc_mask), _ptr(txid), _ptr(eff),
            _ptr(tag), _ptr(add_tok), _ptr(rem_off), _ptr(rem_tok), _ptr(ids), _ptr(due)),
            "agn_oplog_append")
        return ids, due

    def flush(self, stream=None) -> _abi.AgnLog:
        v = _abi.AgnLog()
        check(self.eng.lib.agn_oplog_flush(self.h, C.byref(v), stream), "agn_oplog_flush")
        return v

    def prune(self, prune_ptr, thr_ptr, thr_mask_ptr=None, flags_ptr=None, stream=None):
        check(self.eng.lib.agn_oplog_prune(self.h, prune_ptr, thr_ptr, thr_mask_ptr, flags_ptr,
                                           stream), "agn_oplog_prune")

    def read(self, dreq, dres, stream=None):
        """agn_oplog_read: batched materialize/4 over the resident log (blocks)."""
        rs = dreq.struct if isinstance(dreq, DeviceArrays) else dreq
        os_ = dres.struct if isinstance(dres, DeviceArrays) else dres
        check(self.eng.lib.agn_oplog_read(self.h, C.byref(rs), C.byref(os_), stream),
              "agn_oplog_read")

    def stats(self):
        e, s, t = C.c_uint64(), C.c_uint64(), C.c_uint64()
        check(self.eng.lib.agn_oplog_stats(self.h, C.byref(e), C.byref(s), C.byref(t)))
        return {"entries": e.value, "slots": s.value, "tokens": t.value}

    def gc_due(self, keys):
        """op_insert_gc's GC trigger for the next op of each key (before it is appended)."""
        keys = np.ascontiguousarray(np.atleast_1d(keys), np.uint64)
        out = np.zeros(len(keys), np.uint8)
        check(self.eng.lib.agn_oplog_gc_due(self.h, len(keys), _ptr(keys), _ptr(out)),
              "agn_oplog_gc_due")
        return out.astype(bool)

    def set_counter(self, keys, counters):
        """agn_oplog_set_counter: each key's op counter (the next op gets
        counter + 1) -- one counter per key across several logs."""
        keys = np.ascontiguousarray(np.atleast_1d(keys), np.uint64)
        ctr = np.ascontiguousarray(np.atleast_1d(counters), np.uint32)
        check(self.eng.lib.agn_oplog_set_counter(self.h, len(keys), _ptr(keys), _ptr(ctr)),
              "agn_oplog_set_counter")

    def key_meta(self, keys=None):
        """Per key: (Length, ListLen, op counter) of the ETS tuple it mirrors."""
        keys = np.arange(self.n_keys, dtype=np.uint64) if keys is None else \
            np.ascontiguousarray(keys, np.uint64)
        n = len(keys)
        ln, ll, ct = (np.zeros(n, np.uint32) for _ in range(3))
        check(self.eng.lib.agn_oplog_key_meta(self.h, n, _ptr(keys), _ptr(ln), _ptr(ll), _ptr(ct)),
              "agn_oplog_key_meta")
        return ln, ll, ct


class Batcher:
    """agn_batcher: per-key materializer_vnode:read/6 calls from many threads
    coalesced into batched kernels.  `read` blocks the calling thread (ctypes
    releases the GIL for the duration)."""

    def __init__(self, oplog: OpLog, max_batch: int = 1024, max_wait_us: int = 0,
                 cached: bool = False, slots: int = 0):
        """cached=True: agn_batcher_create_cached -- each batch is the whole
        read/6 over the batcher's device snapshot cache (counter_pn)."""
        self.oplog, self.lib = oplog, oplog.eng.lib
        self.h = C.c_void_p()
        if cached:
            check(self.lib.agn_batcher_create_cached(oplog.h, slots, max_batch, max_wait_us,
                                                     C.byref(self.h)), "agn_batcher_create_cached")
        else:
            check(self.lib.agn_batcher_create(oplog.h, max_batch, max_wait_us, C.byref(self.h)),
                  "agn_batcher_create")

    def close(self):
        if self.h:
            self.lib.agn_batcher_destroy(self.h)
            self.h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def read(self, key, R, R_mask=None, sct=None, sct_mask=None, txid=0, base_value=0,
             base_tag=None, base_tok=None, out_cap=0, gc=False, capacity_ok=False):
        """One read/6; returns a dict of the key's result.  capacity_ok: an
        AGN_ECAPACITY (the state did not fit out_cap) returns the result with
        "ecapacity": True and out_n = the pairs needed, instead of raising."""
        D = self.oplog.n_dcs
        W = n_words(D)
        arr = lambda a: None if a is None else np.ascontiguousarray(a, np.uint64)  # noqa: E731
        R, R_mask, sct, sct_mask = arr(R), arr(R_mask), arr(sct), arr(sct_mask)
        rd = _abi.AgnKeyRead()
        rd.key, rd.R, rd.R_mask, rd.sct, rd.sct_mask = key, _ptr(R), _ptr(R_mask), _ptr(sct), \
            _ptr(sct_mask)
        rd.txid, rd.base_value = txid, base_value
        rd.flags = _abi.READ_GC if gc else 0
        if base_tag is not None:
            base_tag = np.ascontiguousarray(base_tag, np.uint32)
            base_tok = np.ascontiguousarray(base_tok, np.uint64)
            rd.n_base, rd.base_tag, rd.base_tok = len(base_tag), _ptr(base_tag), _ptr(base_tok)
        ct, ctm = np.zeros(D, np.uint64), np.zeros(W, np.uint64)
        otag, otok = np.zeros(max(out_cap, 1), np.uint32), np.zeros(max(out_cap, 1), np.uint64)
        o = _abi.AgnKeyResult()
        o.lastct, o.lastct_mask, o.out_cap = ct.ctypes.data, ctm.ctypes.data, out_cap
        o.out_tag, o.out_tok = otag.ctypes.data, otok.ctypes.data
        rc = self.lib.agn_batcher_read(self.h, C.byref(rd), C.byref(o))
        if rc == _abi.ECAPACITY and capacity_ok:
            return {"ecapacity": True, "out_n": o.out_n, "status": o.status}
        check(rc, "agn_batcher_read")
        return {"value": o.value, "hole": o.hole, "lastct": ct, "lastct_mask": ctm,
                "count": o.count, "flags": o.flags, "err_pos": o.err_pos, "out_n": o.out_n,
                "status": o.status,
                "out_tag": otag[:o.out_n], "out_tok": otok[:o.out_n]}

    def stats(self):
        b, r = C.c_uint64(), C.c_uint64()
        check(self.lib.agn_batcher_stats(self.h, C.byref(b), C.byref(r)))
        return {"batches": b.value, "reads": r.value}

    def state_bound(self, key) -> int:
        """agn_batcher_state_bound: pairs of the largest cached state of key."""
        n = C.c_uint32()
        check(self.lib.agn_batcher_state_bound(self.h, key, C.byref(n)), "agn_batcher_state_bound")
        return n.value

    def store(self, key, clock, clock_mask=None, last_op=0, count=0, value=0, tags=None,
              toks=None, gc=True):
        """agn_batcher_store: materialize_snapshot's store of a snapshot the
        caller materialized from the log (get_from_snapshot_log)."""
        clock = np.ascontiguousarray(clock, np.uint64)
        cm = None if clock_mask is None else np.ascontiguousarray(np.atleast_1d(clock_mask),
                                                                   np.uint64)
        tg = None if tags is None else np.ascontiguousarray(tags, np.uint32)
        tk = None if toks is None else np.ascontiguousarray(toks, np.uint64)
        n = 0 if tg is None else len(tg)
        check(self.lib.agn_batcher_store(self.h, key, _ptr(clock), _ptr(cm), int(last_op),
                                         int(count), int(value), n, _ptr(tg) if n else None,
                                         _ptr(tk) if n else None,
                                         _abi.READ_GC if gc else 0), "agn_batcher_store")


def gen_host(cfg: _abi.AgnGenCfg):
    """Host-generated synthetic log (library-owned arrays) as numpy views."""
    lib = load()
    log, req = _abi.AgnLog(), _abi.AgnRead()
    check(lib.agn_gen_host(C.byref(cfg), C.byref(log), C.byref(req)), "agn_gen_host")
    return log, req


def free_gen_host(log, req):
    load().agn_gen_free_host(C.byref(log), C.byref(req))


def host_view(ptr, dtype, n):
    if not ptr or n == 0:
        return np.zeros(0, dtype)
    ct = np.ctypeslib.as_ctypes_type(np.dtype(dtype))
    return np.ctypeslib.as_array((ct * int(n)).from_address(ptr))


class Interner:
    """agn_interner: exact byte-string <-> dense id map (the NIF's term tables:
    keys, DC ids, TxIds, set elements / register values, tokens).  Host-only."""

    def __init__(self, first_id: int = 1, max_ids: int = 1 << 40):
        self.lib = load()
        self.h = C.c_void_p()
        check(self.lib.agn_interner_create(first_id, max_ids, C.byref(self.h)),
              "agn_interner_create")

    def close(self):
        if self.h:
            self.lib.agn_interner_destroy(self.h)
            self.h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def intern(self, b: bytes):
        """-> (id, is_new)"""
        i, new = C.c_uint64(), C.c_int()
        check(self.lib.agn_intern(self.h, b, len(b), C.byref(i), C.byref(new)), "agn_intern")
        return i.value, bool(new.value)

    def find(self, b: bytes):
        i, f = C.c_uint64(), C.c_int()
        check(self.lib.agn_intern_find(self.h, b, len(b), C.byref(i), C.byref(f)),
              "agn_intern_find")
        return i.value if f.value else None

    def bytes_of(self, i: int) -> bytes:
        p, n = C.c_void_p(), C.c_size_t()
        check(self.lib.agn_intern_bytes(self.h, i, C.byref(p), C.byref(n)), "agn_intern_bytes")
        return C.string_at(p.value, n.value) if n.value else b""

    def __len__(self):
        n = C.c_uint64()
        check(self.lib.agn_interner_size(self.h, C.byref(n)))
        return n.value
