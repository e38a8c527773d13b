"""Host mirror of materializer (src/materializer.erl) over the C ABI.

  create_snapshot(Type)                    :45-47
  update_snapshot(Type, Snapshot, Effect)  :51-58  -> ("ok", S) | ("error", {unexpected_operation, Op, Type})
  materialize_eager(Type, Snapshot, Ops)   :61-70
  belongs_to_snapshot_op(SSTime, {Dc, Ct}, OpSs) :101-106
      (batched form: belongs_to_snapshot_ops — one launch for many ops; both
      evaluate vectorclock:le on the device)
"""
from __future__ import annotations

from . import clocksi_materializer as cm
from .encode import IGNORE, ClocksiPayload
from .records import COUNTER_PN, MaterializedSnapshot, SnapshotGetResponse


def create_snapshot(typ):
    return cm.new(typ)


def update_snapshot(typ, snapshot, effect, device: int = 0):
    r = cm.materialize_eager(typ, snapshot, [effect], device)
    if isinstance(r, tuple) and r and r[0] == "error":
        return r
    return ("ok", r)


def materialize_eager(typ, snapshot, effects, device: int = 0):
    return cm.materialize_eager(typ, snapshot, effects, device)


def belongs_to_snapshot_ops(items, device: int = 0):
    """[(SSTime | "ignore", (OpDc, OpCommitTime), OpSs)] -> [bool]: True when the
    op is NOT covered by SSTime.  Each op becomes a one-op key read with
    R = its own OpSSCommit and SCT = SSTime, so the kernel includes it iff
    notInPrev = not vectorclock:le(OpSSCommit, SSTime)."""
    reads = []
    for ss_time, (dc, ct), op_ss in items:
        oc = dict(op_ss)
        oc[dc] = ct
        p = ClocksiPayload("k", COUNTER_PN, 0, dict(op_ss), (dc, ct), None)
        resp = SnapshotGetResponse([(1, p)], 1, MaterializedSnapshot(0, 0), ss_time, True)
        reads.append((IGNORE, oc, resp))
    out = cm.materialize_batch(COUNTER_PN, reads, device) if reads else []
    return [r[5] == 1 for r in out]


def belongs_to_snapshot_op(ss_time, dc_ct, op_ss, device: int = 0) -> bool:
    return belongs_to_snapshot_ops([(ss_time, dc_ct, op_ss)], device)[0]
