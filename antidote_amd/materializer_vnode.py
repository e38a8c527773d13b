"""Host mirror of materializer_vnode (src/materializer_vnode.erl): the
per-partition op cache (ETS ops tuples) and snapshot cache (vector_orddict),
with its read path, its GC and its resize policy.

  read(Key, Type, SnapshotTime, TxId, _Props, Partition)  :96-102
  update(Key, DownstreamOp)                               :106-110 -> op_insert_gc :621-647
  store_ss(Key, Snapshot, CommitTime)                     :114-118 -> internal_store_ss :341-364

Every vector-clock decision on these paths runs on the device:
materialize/4 (agn_materialize), base-snapshot selection
(vector_orddict:get_smaller -> agn_select_base) and the GC filter of
prune_ops (belongs_to_snapshot_op per cached op, batched into one launch).
The cache bookkeeping itself (tuple slots, list sizes) is host control flow,
as in the reference.
"""
from __future__ import annotations

from . import clocksi_materializer as cm
from .encode import IGNORE
from .materializer import belongs_to_snapshot_ops
from .records import (CorruptedOpsCache, MaterializedSnapshot, OpsTuple,  # noqa: F401
                      SnapshotGetResponse)
from .vector_orddict import VectorOrddict

SNAPSHOT_THRESHOLD = 10  # :37
SNAPSHOT_MIN = 3         # :39
OPS_THRESHOLD = 50       # :41
RESIZE_THRESHOLD = 5     # :44
MIN_OP_STORE_SS = 5      # :47


def _vc_min(a: dict, b: dict) -> dict:
    """vectorclock:min([A, B]) (missing entry = 0)."""
    return {d: min(a.get(d, 0), b.get(d, 0)) for d in set(a) | set(b)}


class LogFallbackRequired(RuntimeError):
    """get_from_snapshot_log (:416-419): no cached snapshot <= the read time;
    the reference reads the partition's disk log (logging_vnode), which is
    outside this engine."""


class MaterializerVnode:
    def __init__(self, partition=0, device: int = 0):
        self.partition = partition
        self.device = device
        self.ops_cache: dict = {}       # key -> OpsTuple
        self.snapshot_cache: dict = {}  # key -> VectorOrddict

    # ------------------------------------------------------------------ API
    def read(self, key, typ, snapshot_time, txid=IGNORE, _props=None):
        return self.internal_read(key, typ, snapshot_time, txid, False)

    def update(self, key, op):
        return self.op_insert_gc(key, op)

    def store_ss(self, key, snapshot: MaterializedSnapshot, commit_time):
        self.internal_store_ss(key, snapshot, commit_time, False)

    # ------------------------------------------------------------------ reads
    def internal_read(self, key, typ, min_snapshot_time, txid, should_gc):
        resp = self.get_from_snapshot_cache(txid, key, typ, min_snapshot_time)
        return self.materialize_snapshot(txid, key, typ, min_snapshot_time, should_gc, resp)

    def get_from_snapshot_cache(self, txid, key, typ, min_snapshot_time):
        if key not in self.snapshot_cache:
            empty = MaterializedSnapshot(0, cm.new(typ))
            self.internal_store_ss(key, empty, {}, False)
            return self._response(((IGNORE, empty), True), key)
        found, is_first = self.snapshot_cache[key].get_smaller(min_snapshot_time, self.device)
        if found is None:
            raise LogFallbackRequired(key)
        return self._response((found, is_first), key)

    def _response(self, found, key):
        (sct, latest), is_first = found
        t = self.ops_cache.get(key)
        ops, n = (t, t.length) if t is not None else ([], 0)
        return SnapshotGetResponse(ops, n, latest, sct, is_first)

    def materialize_snapshot(self, txid, key, typ, snapshot_time, should_gc, resp):
        if resp.number_of_ops == 0:
            return ("ok", resp.materialized_snapshot.value)
        r = cm.materialize(typ, txid, snapshot_time, resp, self.device)
        if r[0] == "error":
            return r
        _, value, new_last_op, commit_time, was_updated, ops_added = r
        if commit_time == IGNORE:
            return ("ok", value)
        refresh = was_updated and resp.is_newest_snapshot and ops_added >= MIN_OP_STORE_SS
        if refresh or should_gc:
            self.internal_store_ss(key, MaterializedSnapshot(new_last_op, value), commit_time,
                                   should_gc)
        return ("ok", value)

    # ------------------------------------------------------------------ snapshot cache + GC
    def internal_store_ss(self, key, snapshot: MaterializedSnapshot, commit_time, should_gc):
        sd = self.snapshot_cache.get(key, VectorOrddict())
        should_insert = True
        if sd.size() > 0:
            should_insert = (snapshot.last_op_id - sd.first()[1].last_op_id) >= MIN_OP_STORE_SS
        if should_insert or should_gc:
            self.snapshot_insert_gc(key, sd.insert_bigger(commit_time, snapshot), should_gc)
            return True
        return False

    def snapshot_insert_gc(self, key, sd: VectorOrddict, should_gc):
        if not (sd.size() >= SNAPSHOT_THRESHOLD or should_gc):
            self.snapshot_cache[key] = sd
            return
        pruned = sd.sublist(1, SNAPSHOT_MIN)
        commit_time = pruned.last()[0]
        for ct1, _ in pruned.to_list():
            commit_time = _vc_min(ct1, commit_time)
        t = self.ops_cache.get(key)
        if t is None:
            t = OpsTuple(key, 0, 0)
        new_ops = self.prune_ops(t, commit_time)
        self.snapshot_cache[key] = pruned
        # prune_ops' NewLength is 1 when nothing survives (:580-583)
        list_len, new_length = t.list_len, max(len(new_ops), 1)
        if new_length > list_len - RESIZE_THRESHOLD:
            new_list_len = list_len * 2
        else:
            half = list_len // 2
            if half <= OPS_THRESHOLD:
                new_list_len = list_len
            elif half - RESIZE_THRESHOLD > new_length:
                new_list_len = half
            else:
                new_list_len = list_len
        self.ops_cache[key] = OpsTuple(key, new_list_len, t.op_counter, new_ops)

    def prune_ops(self, t: OpsTuple, threshold) -> list:
        """Keep the ops not covered by `threshold` (belongs_to_snapshot_op,
        one device launch for the whole tuple)."""
        keep = belongs_to_snapshot_ops(
            [(threshold, p.commit_time, p.snapshot_time) for _i, p in t.ops], self.device)
        # With no survivor the reference stores element(?FIRST_OP+Len), an empty
        # slot of the tuple (0), as the only op (:580-583) -- the next
        # materialize of the key then fails on `{_, Op} = 0`.  The engine
        # (agn_oplog_prune / agn_prune_ops: AGN_GC_ALL_PRUNED) and this mirror
        # keep zero ops instead, and count NewLength as 1 for the resize policy
        # like the reference (intentional deviation).
        return [op for op, k in zip(t.ops, keep) if k]

    # ------------------------------------------------------------------ writes
    def op_insert_gc(self, key, op):
        t = self.ops_cache.get(key)
        if t is None:
            t = self.ops_cache[key] = OpsTuple(key, OPS_THRESHOLD, 0)
        t.op_counter += 1
        new_id = t.op_counter
        if t.length >= t.list_len or new_id % OPS_THRESHOLD == 0:
            self.internal_read(key, op.type, op.snapshot_time, IGNORE, True)
            t = self.ops_cache[key]
            t.op_counter = new_id
        # ets:update_element at slot ?FIRST_OP+Length: the tuple has ListLen+1
        # op slots, one more is badarg in the reference
        if t.length > t.list_len:
            raise RuntimeError(("badarg", "ops tuple full", key))
        t.ops.append((new_id, op))
        return True
