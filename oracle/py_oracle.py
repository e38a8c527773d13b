"""TEST INFRASTRUCTURE ONLY — pure-Python restatement of the reference path.

Used by tests/ to pin the known-answer tests (KATs) of the reference's
EUnit suites and as a second, independent restatement to cross-check the C
oracle (oracle/oracle.c).  Never imported by the product package.

Vector clocks are dicts {dc: int} exactly like the reference's
``dict:dict(dcid(), non_neg_integer())`` (include/antidote.hrl:188); the
vectorclock 0.1.0 predicates read a missing entry as 0.

Restated functions (paths relative to the AntidoteDB tree):
  clocksi_materializer: materialize/4 :89-101, get_first_id/1 :49-63,
      apply_operations/4 :113-121, materialize_intern :157-197,
      is_op_in_snapshot/7 :216-268
  materializer: update_snapshot/3 :51-58, materialize_eager/3 :61-70,
      belongs_to_snapshot_op/3 :101-106
  materializer_vnode: internal_read :371-376, get_from_snapshot_cache :384-413,
      materialize_snapshot :466-509, internal_store_ss :341-364,
      snapshot_insert_gc :515-563, prune_ops :566-585, check_filter :592-604,
      op_insert_gc :621-647 (constants :36-47)
  vector_orddict: :62-183
  stable_time_functions: update_func_min/2 :42-48, get_min_time/1 :51-85
  meta_data_sender: update_stable/3 :341-356
  dc_utilities: get_stable_snapshot/0 (gr branch) :256-277,
      get_scalar_stable_time/0 :295-320
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace
from typing import Any

COUNTER_PN = "antidote_crdt_counter_pn"
SET_AW = "antidote_crdt_set_aw"
REGISTER_MV = "antidote_crdt_register_mv"
IGNORE = "ignore"

FIRST_OP = 4            # include/antidote.hrl:90
SNAPSHOT_THRESHOLD = 10  # src/materializer_vnode.erl:37
SNAPSHOT_MIN = 3         # :39
OPS_THRESHOLD = 50       # :41
RESIZE_THRESHOLD = 5     # :44
MIN_OP_STORE_SS = 5      # :47


class CorruptedOpsCache(Exception):
    """erlang:error(corrupted_ops_cache) (src/clocksi_materializer.erl:191)."""


class BadMatch(Exception):
    """A reference crash path (badmatch / badarg on the ETS tuple)."""


class EtsTuple(list):
    """The ETS ops tuple {Key, {Length, ListLen}, OpCounter, Op1, ...} as a
    1-indexed Python list (element(I, T) == T[I - 1])."""


# ---------------------------------------------------------------- vectorclock
def vc_get(vc: dict, dc) -> int:
    return vc.get(dc, 0)


def vc_le(a: dict, b: dict) -> bool:
    return all(vc_get(a, d) <= vc_get(b, d) for d in set(a) | set(b))


def vc_ge(a: dict, b: dict) -> bool:
    return vc_le(b, a)


def vc_eq(a: dict, b: dict) -> bool:
    return all(vc_get(a, d) == vc_get(b, d) for d in set(a) | set(b))


def vc_gt(a: dict, b: dict) -> bool:
    return vc_ge(a, b) and not vc_eq(a, b)


def vc_conc(a: dict, b: dict) -> bool:
    return not vc_ge(a, b) and not vc_le(a, b)


def vc_all_dots_greater(a: dict, b: dict) -> bool:
    return all(vc_get(a, d) > vc_get(b, d) for d in set(a) | set(b))


def vc_min(vcs: list) -> dict:
    out = dict(vcs[0])
    for v in vcs[1:]:
        out = {d: min(vc_get(out, d), vc_get(v, d)) for d in set(out) | set(v)}
    return out


def vc_max(vcs: list) -> dict:
    out: dict = {}
    for v in vcs:
        out = {d: max(vc_get(out, d), vc_get(v, d)) for d in set(out) | set(v)}
    return out


# ---------------------------------------------------------------- CRDTs
def crdt_new(typ):
    if typ == COUNTER_PN:
        return 0
    if typ in (SET_AW, REGISTER_MV):
        return []
    raise BadMatch(("undef", typ))  # materializer_error_nocreate_test


def crdt_value(typ, state):
    if typ == COUNTER_PN:
        return state
    if typ == SET_AW:
        return [e for e, _ in state]
    if typ == REGISTER_MV:
        return [v for v, _ in state]
    raise BadMatch(("undef", typ))


def crdt_update(typ, effect, state):
    """antidote_crdt_<type>:update/2; raises on a malformed effect."""
    if typ == COUNTER_PN:
        if not isinstance(effect, int) or isinstance(effect, bool):
            raise TypeError("badarith")
        return state + effect
    if typ == SET_AW:
        st = {e: list(toks) for e, toks in state}
        for elem, add, rem in effect:
            toks = [t for t in st.get(elem, []) if t not in rem] + list(add)
            if toks:
                st[elem] = toks
            else:
                st.pop(elem, None)
        return sorted(st.items(), key=lambda kv: kv[0])
    if typ == REGISTER_MV:
        if effect[0] == "reset":
            _, ovr = effect
            return [(v, t) for v, t in state if t not in ovr]
        value, token, ovr = effect
        kept = [(v, t) for v, t in state if t not in ovr]
        return sorted(kept + [(value, token)])
    raise BadMatch(("undef", typ))


def update_snapshot(typ, snapshot, op):
    """materializer:update_snapshot/3: any exception -> error tuple."""
    try:
        return ("ok", crdt_update(typ, op, snapshot))
    except Exception:
        return ("error", ("unexpected_operation", op, typ))


def materialize_eager(typ, snapshot, effects):
    for e in effects:
        r = update_snapshot(typ, snapshot, e)
        if r[0] == "error":
            return r
        snapshot = r[1]
    return snapshot


# ---------------------------------------------------------------- payloads
@dataclass
class Payload:
    """#clocksi_payload{} (include/antidote.hrl:197-204)."""
    key: Any
    type: str
    op_param: Any
    snapshot_time: dict
    commit_time: tuple  # (dc, time)
    txid: Any = None


@dataclass
class MaterializedSnapshot:
    last_op_id: int
    value: Any


@dataclass
class SnapshotGetResponse:
    ops_list: Any            # list [(id, payload)] newest first, or an ETS tuple (list)
    number_of_ops: int
    materialized_snapshot: MaterializedSnapshot
    snapshot_time: Any       # dict or IGNORE
    is_newest_snapshot: bool = True


def belongs_to_snapshot_op(ss_time, dc_ct, op_ss) -> bool:
    if ss_time == IGNORE:
        return True
    dc, ct = dc_ct
    op_ss1 = dict(op_ss)
    op_ss1[dc] = ct
    return not vc_le(op_ss1, ss_time)


def is_op_in_snapshot(txid, op: Payload, dc_ct, op_ss, snapshot_time, last_snapshot,
                      prev_time):
    if belongs_to_snapshot_op(last_snapshot, dc_ct, op_ss) or (txid == op.txid):
        dc, ct = dc_ct
        oc = dict(op_ss)
        oc[dc] = ct
        prev2 = oc if prev_time == IGNORE else prev_time
        result, new_time = True, dict(prev2)
        for d, t in oc.items():
            if d in snapshot_time:
                if snapshot_time[d] < t:
                    result = False
            else:
                result = False  # logger:error("Could not find DC in SS")
            new_time[d] = max(new_time[d], t) if d in new_time else t
        return (True, False, new_time) if result else (False, False, prev_time)
    return (False, True, prev_time)


def _tuple_len(tup):
    return tup[1][0]


def get_first_id(ops) -> int:
    if not isinstance(ops, EtsTuple):
        return ops[0][0] if ops else 0
    length = _tuple_len(ops)
    if length == 0:
        return 0
    el = ops[FIRST_OP + length - 1 - 1]
    if not isinstance(el, tuple):
        raise BadMatch(el)
    return el[0]


def materialize_intern(typ, op_list, last_op, first_hole, sct, min_snapshot_time, ops,
                       txid, last_op_ct, new_ss, location=0):
    if not isinstance(ops, EtsTuple):
        seq = ops
    else:
        length = _tuple_len(ops)
        seq = []
        for loc in range(length):
            el = ops[(FIRST_OP + length - 1) - loc - 1]
            if not isinstance(el, tuple):
                raise BadMatch(el)
            seq.append(el)
    for op_id, op in seq:
        if typ != op.type:
            raise CorruptedOpsCache()
        incl, in_prev, new_ct = is_op_in_snapshot(txid, op, op.commit_time,
                                                  op.snapshot_time, min_snapshot_time,
                                                  sct, last_op_ct)
        if incl:
            op_list = [op] + op_list
            last_op_ct, new_ss = new_ct, True
        elif not in_prev:
            first_hole = op_id - 1
    return ("ok", op_list, first_hole, last_op_ct, new_ss)


def apply_operations(typ, snapshot, count, op_list):
    for op in op_list:
        r = update_snapshot(typ, snapshot, op.op_param)
        if r[0] == "error":
            return r
        snapshot, count = r[1], count + 1
    return ("ok", snapshot, count)


def materialize(typ, txid, min_snapshot_time, resp: SnapshotGetResponse):
    """clocksi_materializer:materialize/4 ->
    ("ok", Value, NewLastOp, LastOpCt, IsNewSS, Count) | ("error", Reason)."""
    sct = resp.snapshot_time
    ops = resp.ops_list
    first_id = get_first_id(ops)
    _, op_list, new_last_op, last_op_ct, is_new_ss = materialize_intern(
        typ, [], resp.materialized_snapshot.last_op_id, first_id, sct,
        min_snapshot_time, ops, txid, sct, False)
    r = apply_operations(typ, resp.materialized_snapshot.value, 0, op_list)
    if r[0] == "error":
        return r
    return ("ok", r[1], new_last_op, last_op_ct, is_new_ss, r[2])


# ---------------------------------------------------------------- vector_orddict
class VectorOrddict:
    """{[{VC, Val}], Size}, newest first (src/vector_orddict.erl:36-43)."""

    def __init__(self, lst=None):
        self.lst = list(lst or [])

    def size(self):
        return len(self.lst)

    def get_smaller(self, vector):
        is_first = True
        for clock, val in self.lst:
            if vc_le(clock, vector):
                return (clock, val), is_first
            is_first = False
        return None, is_first

    def get_smaller_from_id(self, dc, time):
        for clock, val in self.lst:
            if vc_get(clock, dc) <= time:
                return clock, val
        return None

    def insert(self, vector, val):
        for i, (clock, _) in enumerate(self.lst):
            if vc_all_dots_greater(vector, clock):
                return VectorOrddict(self.lst[:i] + [(vector, val)] + self.lst[i:])
        return VectorOrddict(self.lst + [(vector, val)])

    def insert_bigger(self, vector, val):
        if not self.lst:
            return VectorOrddict([(vector, val)])
        if not vc_le(vector, self.lst[0][0]):
            return VectorOrddict([(vector, val)] + self.lst)
        return VectorOrddict(self.lst)

    def sublist(self, start, length):
        return VectorOrddict(self.lst[start - 1:start - 1 + length])

    def first(self):
        return self.lst[0]

    def last(self):
        return self.lst[-1]

    def filter(self, fun):
        return VectorOrddict([x for x in self.lst if fun(x)])

    def is_concurrent_with_any(self, other):
        return any(vc_conc(c, other) for c, _ in self.lst)


# ---------------------------------------------------------------- materializer_vnode
class MaterializerVnode:
    """ETS-backed state of one partition: ops_cache (key -> ops tuple as a
    1-indexed Python list) and snapshot_cache (key -> VectorOrddict).
    disk_log=True also models the partition's logging_vnode disk log (every
    committed payload, commit order), which get_from_snapshot_log reads;
    without it that fallback raises NotImplementedError."""

    def __init__(self, disk_log: bool = False):
        self.ops_cache: dict = {}
        self.snapshot_cache: dict = {}
        self.disk_log: list | None = [] if disk_log else None

    # -- reads
    def internal_read(self, key, typ, min_snapshot_time, txid, should_gc):
        resp = self.get_from_snapshot_cache(txid, key, typ, min_snapshot_time)
        return self.materialize_snapshot(txid, key, typ, min_snapshot_time, should_gc, resp)

    def read(self, key, typ, snapshot_time, txid):
        return self.internal_read(key, typ, snapshot_time, txid, False)

    def get_from_snapshot_cache(self, txid, key, typ, min_snapshot_time):
        if key not in self.snapshot_cache:
            empty = MaterializedSnapshot(0, crdt_new(typ))
            self.store_snapshot(txid, key, empty, {}, False)
            return self.update_snapshot_from_cache(((IGNORE, empty), True), key)
        found, is_first = self.snapshot_cache[key].get_smaller(min_snapshot_time)
        if found is None:
            return self.get_from_snapshot_log(key, typ, min_snapshot_time)
        return self.update_snapshot_from_cache((found, is_first), key)

    def get_from_snapshot_log(self, key, typ, snapshot_time):
        """get_from_snapshot_log (:416-419) -> logging_vnode:get_up_to_time
        (src/logging_vnode.erl:185-190) -> {get, LogId, undefined, Max, Type,
        Key} (:522-549): the key's committed ops whose transaction snapshot
        passes check_max_time (vectorclock:le(SnapshotTime, Max), :778-779),
        in log order, then reverse_and_add_op_id (:586-591): newest first,
        ids from 0 at the oldest; base {last_op_id 0, Type:new()},
        snapshot_time vectorclock:new(), is_newest_snapshot false."""
        if self.disk_log is None:
            raise NotImplementedError("get_from_snapshot_log (logging_vnode fallback)")
        ops = [p for p in self.disk_log if p.key == key and vc_le(p.snapshot_time, snapshot_time)]
        newest_first = [(i, p) for i, p in enumerate(ops)][::-1]
        return SnapshotGetResponse(newest_first, len(ops), MaterializedSnapshot(0, crdt_new(typ)),
                                   {}, False)

    def store_snapshot(self, txid, key, snapshot, time, should_gc):
        self.internal_store_ss(key, snapshot, time, should_gc)

    def update_snapshot_from_cache(self, resp, key):
        (sct, latest), is_first = resp
        ops, n = self.fetch_updates_from_cache(key)
        return SnapshotGetResponse(ops, n, latest, sct, is_first)

    def fetch_updates_from_cache(self, key):
        if key not in self.ops_cache:
            return [], 0
        tup = self.ops_cache[key]
        return tup, tup[1][0]

    def materialize_snapshot(self, txid, key, typ, snapshot_time, should_gc,
                             resp: SnapshotGetResponse):
        if resp.number_of_ops == 0:
            return ("ok", resp.materialized_snapshot.value)
        r = materialize(typ, txid, snapshot_time, resp)
        if r[0] == "error":
            return r
        _, value, new_last_op, commit_time, was_updated, ops_added = r
        if commit_time == IGNORE:
            return ("ok", value)
        refresh = was_updated and resp.is_newest_snapshot and ops_added >= MIN_OP_STORE_SS
        if refresh or should_gc:
            self.store_snapshot(txid, key, MaterializedSnapshot(new_last_op, value),
                                commit_time, should_gc)
        return ("ok", value)

    # -- snapshot cache + GC
    def internal_store_ss(self, key, snapshot: MaterializedSnapshot, commit_time, should_gc):
        sd = self.snapshot_cache.get(key, VectorOrddict())
        if sd.size() > 0:
            should_insert = (snapshot.last_op_id - sd.first()[1].last_op_id) >= MIN_OP_STORE_SS
        else:
            should_insert = True
        if should_insert or should_gc:
            sd1 = sd.insert_bigger(commit_time, snapshot)
            self.snapshot_insert_gc(key, sd1, should_gc)
            return True
        return False

    def snapshot_insert_gc(self, key, sd: VectorOrddict, should_gc):
        if sd.size() >= SNAPSHOT_THRESHOLD or should_gc:
            pruned = sd.sublist(1, SNAPSHOT_MIN)
            ct, _ = pruned.last()
            commit_time = ct
            for ct1, _ in pruned.lst:
                commit_time = vc_min([ct1, commit_time])
            if key in self.ops_cache:
                tup = self.ops_cache[key]
                length, list_len = tup[1]
                op_id = tup[2]
            else:
                tup, length, op_id, list_len = EtsTuple(), 0, 0, 0
            new_length, pruned_ops = self.prune_ops(length, tup, commit_time)
            self.snapshot_cache[key] = pruned
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
            new_tup = EtsTuple([0] * (FIRST_OP + new_list_len))
            new_tup[0] = key
            new_tup[1] = (new_length, new_list_len)
            new_tup[2] = op_id
            for pos, el in pruned_ops:
                new_tup[pos - 1] = el
            self.ops_cache[key] = new_tup
        else:
            self.snapshot_cache[key] = sd

    @staticmethod
    def prune_ops(length, tup, threshold):
        new_size, new_ops, new_id = 0, [], FIRST_OP
        for idx in range(FIRST_OP, FIRST_OP + length):
            el = tup[idx - 1]
            _op_id, op = el
            if belongs_to_snapshot_op(threshold, op.commit_time, op.snapshot_time):
                new_ops.append((new_id, el))
                new_id += 1
                new_size += 1
        if new_size == 0:
            idx = FIRST_OP + length
            if idx - 1 >= len(tup):
                raise BadMatch("badarg element/2")
            return 1, [(FIRST_OP, tup[idx - 1])]
        return new_size, new_ops

    # -- writes
    def update(self, key, op: Payload):
        # the commit is logged before the materializer sees the op
        # (clocksi_vnode:commit -> logging_vnode:append_commit, then
        # update_materializer, src/clocksi_vnode.erl:499-528,636-656)
        if self.disk_log is not None:
            self.disk_log.append(op)
        return self.op_insert_gc(key, op)

    def op_insert_gc(self, key, op: Payload):
        if key not in self.ops_cache:
            tup = EtsTuple([0] * (FIRST_OP + OPS_THRESHOLD))
            tup[0] = key
            tup[1] = (0, OPS_THRESHOLD)
            self.ops_cache[key] = tup
        tup = self.ops_cache[key]
        tup[2] += 1
        new_id = tup[2]
        length, list_len = tup[1]
        if length >= list_len or new_id % OPS_THRESHOLD == 0:
            self.internal_read(key, op.type, op.snapshot_time, IGNORE, True)
            tup = self.ops_cache[key]
            new_length, new_list_len = tup[1]
            pos = new_length + FIRST_OP
            if pos - 1 >= len(tup):
                raise BadMatch("badarg update_element")
            tup[pos - 1] = (new_id, op)
            tup[1] = (new_length + 1, new_list_len)
        else:
            pos = length + FIRST_OP
            if pos - 1 >= len(tup):
                raise BadMatch("badarg update_element")
            tup[pos - 1] = (new_id, op)
            tup[1] = (length + 1, list_len)
        return True


# ---------------------------------------------------------------- stable time
UNDEFINED = "undefined"


def get_min_time(d: dict) -> dict:
    """stable_time_functions:get_min_time/1: d maps node/partition -> dict | UNDEFINED."""
    min_dict: dict = {}
    found_undefined = False
    for _node, node_dict in d.items():
        if node_dict == UNDEFINED or node_dict is None:
            found_undefined = True
            continue
        for dc, t in node_dict.items():
            prev = min_dict.get(dc, t)
            min_dict[dc] = t if prev >= t else prev
    if found_undefined:
        return {dc: 0 for dc in min_dict}
    return min_dict


def update_func_min(last, time) -> bool:
    return True if last is None else time >= last


def update_stable(last_result: dict, new_dict: dict, update_func=update_func_min):
    changed, acc = False, dict(last_result)
    for dc, t in new_dict.items():
        if update_func(last_result.get(dc), t):
            changed, acc[dc] = True, t
    return changed, acc


def gst_exchange(local_partition_dicts: list, remote_node_dicts: list) -> dict:
    """meta_data_sender send_meta_data (:230-255): local_merged = min over the
    local partitions, then min over {local_merged} U remote node dicts."""
    local_merged = get_min_time({i: p for i, p in enumerate(local_partition_dicts)})
    allm = {"local_merged": local_merged}
    allm.update({("n", i): r for i, r in enumerate(remote_node_dicts)})
    return get_min_time(allm)


def scalar_stable_time(ss: dict):
    """dc_utilities gr branch: GST = lists:min(values), replicated to every DC."""
    if not ss:
        return ss
    g = min(ss.values())
    return {dc: g for dc in ss}


# ---------------------------------------------------------------- inter-DC dependency check
def vc_set_clock_of_dc(dc, t, vc: dict) -> dict:
    out = dict(vc)
    out[dc] = t
    return out


def dependencies_satisfied(origin_dc, txn_snapshot: dict, partition_clock: dict) -> bool:
    """inter_dc_dep_vnode:try_store/2 (src/inter_dc_dep_vnode.erl:128-155):
    Dependencies = set_clock_of_dc(DCID, 0, Snapshot), CurrentClock =
    set_clock_of_dc(DCID, 0, PartitionClock), applicable iff
    vectorclock:ge(CurrentClock, Dependencies)."""
    deps = vc_set_clock_of_dc(origin_dc, 0, txn_snapshot)
    cur = vc_set_clock_of_dc(origin_dc, 0, partition_clock)
    return vc_ge(cur, deps)
