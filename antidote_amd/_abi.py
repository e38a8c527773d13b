"""ctypes mirror of include/antidote_gpu.h (structs, constants, prototypes).

Shared by the product loader (antidote_amd._lib) and by the test harness,
which binds the same struct layout to the CPU oracle (oracle/liboracle.so).
"""
from __future__ import annotations

import ctypes as C

ABI_VERSION = 6

OK = 0
EINVAL, EHIP, ENOMEM, ECAPACITY, ENOTSUP, ERCCL, ENODEV = -1, -2, -3, -4, -5, -6, -7

COUNTER_PN, SET_AW, REGISTER_MV = 1, 2, 3
TYPE_MIXED = 0xFF
EFFECT_INVALID = -(1 << 63)
TAG_INVALID = 0xFFFFFFFF

F_NEWSS, F_CT_IGNORE, F_ERR_UNEXPECTED, F_ERR_CORRUPTED, F_ERR_CAPACITY = 0x1, 0x2, 0x4, 0x8, 0x10
F_CT_FULL = 0x20          # ABI v5: LastOpCt has every column (mask not written)
HINT_R_FULL, HINT_CT_FLAG, HINT_MIXED = 0x1, 0x2, 0x4
OPS_THRESHOLD = 50  # src/materializer_vnode.erl:41
RESIZE_THRESHOLD = 5  # :44
GC_ALL_PRUNED = 0x1
UNIQUE_ID_BYTES = 128
U64_MAX = (1 << 64) - 1

TYPE_NAMES = {
    COUNTER_PN: "antidote_crdt_counter_pn",
    SET_AW: "antidote_crdt_set_aw",
    REGISTER_MV: "antidote_crdt_register_mv",
}
TYPE_IDS = {v: k for k, v in TYPE_NAMES.items()}

P = C.c_void_p


class AgnLog(C.Structure):
    _fields_ = [
        ("crdt_type", C.c_uint32), ("n_dcs", C.c_uint32),
        ("n_keys", C.c_uint64), ("n_entries", C.c_uint64),
        ("key_off", P), ("key_len", P), ("key_type", P), ("oc", P), ("oc_mask", P),
        ("op_id", P), ("txid", P), ("eff", P),
        ("tag", P), ("add_tok", P), ("rem_off", P), ("rem_tok", P),
        ("key_id0", P), ("key_mask", P),
    ]


ID0_NONE = 0xFFFFFFFF


class AgnRead(C.Structure):
    _fields_ = [
        ("n_req", C.c_uint64), ("keys", P), ("R", P), ("R_mask", P),
        ("sct", P), ("sct_mask", P), ("sct_ignore", P), ("txid", P),
        ("req_type", C.c_uint32), ("hints", C.c_uint32),
        ("base_value", P), ("base_off", P), ("base_tag", P), ("base_tok", P),
    ]


class AgnResult(C.Structure):
    _fields_ = [
        ("value", P), ("hole", P), ("lastct", P), ("lastct_mask", P),
        ("count", P), ("flags", P), ("err_pos", P),
        ("out_off", P), ("out_n", P), ("out_tag", P), ("out_tok", P),
    ]


class AgnSsCache(C.Structure):
    _fields_ = [
        ("n_dcs", C.c_uint32), ("slots", C.c_uint32), ("n_keys", C.c_uint64),
        ("n", P), ("clock", P), ("clock_mask", P), ("last_op", P), ("value", P),
        ("state_tag", P), ("state_tok", P), ("state_cap", C.c_uint64), ("state_ctl", P),
    ]


def ss_state(start, pairs):
    """AGN_SS_STATE(start, pairs): a snapshot state in a cache's arena."""
    return (start << 24) | pairs


def ss_state_unpack(v):
    v &= (1 << 64) - 1
    return v >> 24, v & 0xFFFFFF


class AgnKeyRead(C.Structure):
    _fields_ = [
        ("key", C.c_uint64), ("R", P), ("R_mask", P), ("sct", P), ("sct_mask", P),
        ("txid", C.c_uint64), ("base_value", C.c_int64), ("n_base", C.c_uint32),
        ("flags", C.c_uint32), ("base_tag", P), ("base_tok", P),
    ]


class AgnKeyResult(C.Structure):
    _fields_ = [
        ("value", C.c_int64), ("hole", C.c_int64), ("lastct", P), ("lastct_mask", P),
        ("count", C.c_uint32), ("flags", C.c_uint32), ("err_pos", C.c_uint32),
        ("out_cap", C.c_uint32), ("out_n", C.c_uint32), ("status", C.c_uint32),
        ("out_tag", P), ("out_tok", P),
    ]


class AgnLogRecords(C.Structure):
    _fields_ = [
        ("n", C.c_uint64), ("kind", P), ("txid", P), ("key", P), ("commit_dc", P),
        ("commit_time", P), ("ss", P), ("ss_mask", P), ("eff", P), ("tag", P), ("add_tok", P),
        ("rem_off", P), ("rem_tok", P),
    ]


REC_OTHER, REC_UPDATE, REC_COMMIT = 0, 1, 2
SNAPSHOT_THRESHOLD, SNAPSHOT_MIN, MIN_OP_STORE_SS = 10, 3, 5
SS_HIT, SS_NEW, SS_LOG = 0, 1, 2
READ_GC = 0x1


class AgnGenCfg(C.Structure):
    _fields_ = [
        ("crdt_type", C.c_uint32), ("n_dcs", C.c_uint32), ("n_keys", C.c_uint64),
        ("ops_per_key", C.c_uint32), ("n_elems", C.c_uint32), ("seed", C.c_uint64),
        ("key_base", C.c_uint64), ("key_stride", C.c_uint64),
        ("warm", C.c_uint32), ("_pad", C.c_uint32),
    ]


# Every symbol include/antidote_gpu.h declares, with its ctypes signature.
PROTOTYPES = {
    "agn_abi_version": (C.c_int, []),
    "agn_last_error": (C.c_char_p, []),
    "agn_env_reload": (C.c_int, []),
    "agn_strerror": (C.c_char_p, [C.c_int]),
    "agn_open": (C.c_int, [C.c_int, C.POINTER(P)]),
    "agn_close": (C.c_int, [P]),
    "agn_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "agn_pool_trim": (C.c_int, [P, C.c_uint64]),
    "agn_dev_alloc": (C.c_int, [P, C.c_size_t, C.POINTER(P)]),
    "agn_dev_free": (C.c_int, [P, P]),
    "agn_memcpy_h2d": (C.c_int, [P, P, P, C.c_size_t, P]),
    "agn_memcpy_d2h": (C.c_int, [P, P, P, C.c_size_t, P]),
    "agn_memset_d": (C.c_int, [P, P, C.c_int, C.c_size_t, P]),
    "agn_stream_sync": (C.c_int, [P, P]),
    "agn_materialize": (C.c_int, [P, C.POINTER(AgnLog), C.POINTER(AgnRead),
                                  C.POINTER(AgnResult), P]),
    "agn_materialize_host": (C.c_int, [P, C.POINTER(AgnLog), C.POINTER(AgnRead),
                                       C.POINTER(AgnResult)]),
    "agn_state_capacity": (C.c_int, [C.POINTER(AgnLog), C.POINTER(AgnRead), P]),
    "agn_log_index_ids": (C.c_int, [P, C.POINTER(AgnLog), P, P]),
    "agn_log_index_masks": (C.c_int, [P, C.POINTER(AgnLog), P, P]),
    "agn_tune": (C.c_int, [P, C.POINTER(AgnLog), C.POINTER(AgnRead), C.POINTER(AgnResult), P,
                           C.c_int, C.POINTER(C.c_int), P]),
    "agn_select_base": (C.c_int, [P, C.c_uint32, C.c_uint64, P, P, P, P, P, P, P, P]),
    "agn_gst_min": (C.c_int, [P, C.c_uint32, C.c_uint64, C.c_uint64, P, P, P, P]),
    "agn_gst_finalize": (C.c_int, [P, C.c_uint32, C.c_uint64, P, P]),
    "agn_update_stable": (C.c_int, [C.c_uint32, P, P, C.POINTER(C.c_int)]),
    "agn_log_ingest": (C.c_int, [P, C.POINTER(AgnLogRecords), C.c_uint32, C.c_uint32,
                                 C.c_uint64, P, P, C.c_uint32, C.POINTER(AgnLog), P, P]),
    "agn_ss_lookup": (C.c_int, [P, C.POINTER(AgnSsCache), C.c_uint64, P, P, P, P, P, P, P, P,
                                P, P]),
    "agn_ss_store": (C.c_int, [P, C.POINTER(AgnSsCache), C.POINTER(AgnLog), C.c_uint64, P, P, P,
                               P, C.POINTER(AgnResult), P, P, P, P, P]),
    "agn_ss_state_compact": (C.c_int, [P, C.POINTER(AgnSsCache), P, P, C.c_uint64, P]),
    "agn_read_cached": (C.c_int, [P, C.POINTER(AgnSsCache), C.POINTER(AgnLog), C.c_uint64, P, P,
                                  P, P, C.POINTER(AgnResult), P, P, P, P]),
    "agn_prune_ops": (C.c_int, [P, C.POINTER(AgnLog), P, P, P, C.POINTER(AgnLog), P, P, P]),
    "agn_gst_scalar": (C.c_int, [P, C.c_uint32, C.c_uint64, P, P, P]),
    "agn_oplog_create": (C.c_int, [P, C.c_uint32, C.c_uint32, C.c_uint64, C.c_int, C.c_uint32,
                                   C.POINTER(P)]),
    "agn_oplog_destroy": (C.c_int, [P]),
    "agn_oplog_append": (C.c_int, [P, C.c_uint64, P, P, P, P, P, P, P, P, P, P, P, P]),
    "agn_oplog_flush": (C.c_int, [P, C.POINTER(AgnLog), P]),
    "agn_oplog_prune": (C.c_int, [P, P, P, P, P, P]),
    "agn_oplog_read": (C.c_int, [P, C.POINTER(AgnRead), C.POINTER(AgnResult), P]),
    "agn_batcher_create": (C.c_int, [P, C.c_uint32, C.c_uint32, C.POINTER(P)]),
    "agn_batcher_destroy": (C.c_int, [P]),
    "agn_batcher_read": (C.c_int, [P, C.POINTER(AgnKeyRead), C.POINTER(AgnKeyResult)]),
    "agn_batcher_stats": (C.c_int, [P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "agn_batcher_state_bound": (C.c_int, [P, C.c_uint64, C.POINTER(C.c_uint32)]),
    "agn_batcher_store": (C.c_int, [P, C.c_uint64, P, P, C.c_int64, C.c_uint32, C.c_int64,
                                    C.c_uint32, P, P, C.c_uint32]),
    "agn_batcher_create_cached": (C.c_int, [P, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(P)]),
    "agn_oplog_stats": (C.c_int, [P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                  C.POINTER(C.c_uint64)]),
    "agn_oplog_key_meta": (C.c_int, [P, C.c_uint64, P, P, P, P]),
    "agn_oplog_gc_due": (C.c_int, [P, C.c_uint64, P, P]),
    "agn_oplog_set_counter": (C.c_int, [P, C.c_uint64, P, P]),
    "agn_interner_create": (C.c_int, [C.c_uint64, C.c_uint64, C.POINTER(P)]),
    "agn_interner_destroy": (C.c_int, [P]),
    "agn_intern": (C.c_int, [P, P, C.c_size_t, C.POINTER(C.c_uint64), C.POINTER(C.c_int)]),
    "agn_intern_find": (C.c_int, [P, P, C.c_size_t, C.POINTER(C.c_uint64), C.POINTER(C.c_int)]),
    "agn_intern_bytes": (C.c_int, [P, C.c_uint64, C.POINTER(P), C.POINTER(C.c_size_t)]),
    "agn_interner_size": (C.c_int, [P, C.POINTER(C.c_uint64)]),
    "agn_dep_check": (C.c_int, [P, C.c_uint32, C.c_uint64, P, P, P, P, C.c_uint64, P, P, P, P]),
    "agn_comm_unique_id": (C.c_int, [P]),
    "agn_comm_init": (C.c_int, [P, C.c_int, C.c_int, P]),
    "agn_comm_destroy": (C.c_int, [P]),
    "agn_gst_allreduce": (C.c_int, [P, P, C.c_uint64, P]),
    "agn_gst_merge": (C.c_int, [C.c_uint32, C.c_uint64, P, P]),
    "agn_gen_host": (C.c_int, [C.POINTER(AgnGenCfg), C.POINTER(AgnLog), C.POINTER(AgnRead)]),
    "agn_gen_free_host": (C.c_int, [C.POINTER(AgnLog), C.POINTER(AgnRead)]),
    "agn_gen_dev": (C.c_int, [P, C.POINTER(AgnGenCfg), C.POINTER(AgnLog),
                              C.POINTER(AgnRead), P]),
    "agn_gen_free_dev": (C.c_int, [P, C.POINTER(AgnLog), C.POINTER(AgnRead)]),
}

ORACLE_PROTOTYPES = {
    "oracle_materialize": (C.c_int, [C.POINTER(AgnLog), C.POINTER(AgnRead),
                                     C.POINTER(AgnResult), C.c_int]),
    "oracle_gst_min": (C.c_int, [C.c_uint32, C.c_uint64, C.c_uint64, P, P, P, C.c_int]),
    "oracle_update_stable": (C.c_int, [C.c_uint32, P, P, C.POINTER(C.c_int)]),
    "oracle_select_base": (C.c_int, [C.c_uint32, C.c_uint64, P, P, P, P, P, P, P]),
    "oracle_log_ingest": (C.c_int, [C.POINTER(AgnLogRecords), C.c_uint32, C.c_uint32,
                                    C.c_uint64, P, P, C.c_uint32, C.POINTER(AgnLog)]),
    "oracle_ss_lookup": (C.c_int, [C.POINTER(AgnSsCache), C.c_uint64, P, P, P, P, P, P, P, P,
                                   P]),
    "oracle_ss_store": (C.c_int, [C.POINTER(AgnSsCache), C.POINTER(AgnLog), C.c_uint64, P, P,
                                  P, P, C.POINTER(AgnResult), P, P, P, P]),
    "oracle_prune_ops": (C.c_int, [C.POINTER(AgnLog), P, P, P, C.POINTER(AgnLog), P]),
    "oracle_gst_scalar": (C.c_int, [C.c_uint32, C.c_uint64, P, P]),
    "oracle_dep_check": (C.c_int, [C.c_uint32, C.c_uint64, P, P, P, P, C.c_uint64, P, P, P]),
    "oracle_vc_le": (C.c_int, [C.c_uint32, P, P, P, P]),
    "oracle_vc_all_dots_greater": (C.c_int, [C.c_uint32, P, P, P, P]),
}


def bind(lib, protos):
    for name, (res, args) in protos.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib
