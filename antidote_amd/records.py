"""Records of include/antidote.hrl used at the materializer boundary."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any

from .encode import IGNORE, ClocksiPayload  # noqa: F401  (#clocksi_payload{}, :197-204)

COUNTER_PN = "antidote_crdt_counter_pn"
SET_AW = "antidote_crdt_set_aw"
REGISTER_MV = "antidote_crdt_register_mv"
FIRST_OP = 4  # include/antidote.hrl:90


class CorruptedOpsCache(Exception):
    """erlang:error(corrupted_ops_cache) (src/clocksi_materializer.erl:190-191)."""


@dataclass
class MaterializedSnapshot:
    """#materialized_snapshot{last_op_id, value} (include/antidote.hrl:169-176)."""
    last_op_id: int
    value: Any


@dataclass
class SnapshotGetResponse:
    """#snapshot_get_response{} (include/antidote.hrl:255-266).  ops_list is
    [(op_id, ClocksiPayload)] newest first, or an OpsTuple (ETS form)."""
    ops_list: Any
    number_of_ops: int
    materialized_snapshot: MaterializedSnapshot
    snapshot_time: Any = IGNORE
    is_newest_snapshot: bool = True


class OpsTuple:
    """The ETS ops tuple {Key, {Length, ListLen}, OpCounter, Op1..OpN, 0...}
    (src/materializer_vnode.erl:612-618, include/antidote.hrl:81-90): ops are
    stored oldest first from slot ?FIRST_OP."""

    def __init__(self, key, list_len: int, op_counter: int = 0, ops=None):
        self.key = key
        self.list_len = list_len
        self.op_counter = op_counter
        self.ops = list(ops or [])  # [(op_id, payload)] oldest first; len == Length

    @property
    def length(self):
        return len(self.ops)

    def newest_first(self):
        return list(reversed(self.ops))


def ops_oldest_first(ops_list) -> list:
    if isinstance(ops_list, OpsTuple):
        return list(ops_list.ops)
    return list(reversed(ops_list))
