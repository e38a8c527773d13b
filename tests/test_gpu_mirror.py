"""The reference's own known-answer tests, run through the host mirror of its
Erlang interface (antidote_amd.clocksi_materializer / materializer /
materializer_vnode / vector_orddict / stable_time_functions) — i.e. through
the HIP engine — so they read like the EUnit suites they transcribe."""
import pytest

from antidote_amd import clocksi_materializer as cm
from antidote_amd import materializer, stable_time_functions
from antidote_amd.encode import IGNORE, ClocksiPayload
from antidote_amd.materializer_vnode import MaterializerVnode
from antidote_amd.records import CorruptedOpsCache, MaterializedSnapshot, SnapshotGetResponse
from antidote_amd.vector_orddict import VectorOrddict
from kat_util import TYPES, effect_of, kats, system_seq_log, to_vc

pytestmark = pytest.mark.gpu


def payload(p, typ):
    return ClocksiPayload("k", typ, effect_of(p), to_vc(p["ss"]), tuple(p["ct"]), p["tx"])


def ops_of(c):
    typ = TYPES[c["type"]]
    return [(i, payload(p, typ)) for i, p in c["ops"]]


MAT = kats({"materialize", "materialize_chain"})


@pytest.mark.parametrize("c", MAT, ids=[c["name"] for c in MAT])
def test_materialize_kat(c):
    typ = TYPES[c["type"]]
    ops = ops_of(c)
    if c["kind"] == "materialize_chain":
        f = c["first"]
        r1 = cm.materialize(typ, IGNORE, to_vc(f["R"]), SnapshotGetResponse(
            ops, len(ops), MaterializedSnapshot(*f["base"]), to_vc(f["sct"])))
        _, v1, hole1, ct1, _, _ = r1
        r = cm.materialize(typ, IGNORE, to_vc(c["R"]), SnapshotGetResponse(
            ops, len(ops), MaterializedSnapshot(hole1, v1), ct1))
    else:
        r = cm.materialize(typ, IGNORE, to_vc(c["R"]), SnapshotGetResponse(
            ops, len(ops), MaterializedSnapshot(*c["base"]), to_vc(c["sct"])))
    e = c["expect"]
    assert r[0] == "ok"
    if "value" in e:
        assert cm.value(typ, r[1]) == e["value"]
    if "hole" in e:
        assert r[2] == e["hole"]
    if "ct" in e:
        assert r[3] == (IGNORE if e["ct"] is None else to_vc(e["ct"]))


EAGER = kats({"eager"})


@pytest.mark.parametrize("c", EAGER, ids=[c["name"] for c in EAGER])
def test_eager_kat(c):
    typ = TYPES[c["type"]]
    effs = [tuple(e.values()) if isinstance(e, dict) else e for e in c["effects"]]
    r = materializer.materialize_eager(typ, materializer.create_snapshot(typ), effs)
    if "error" in c["expect"]:
        assert r == ("error", ("unexpected_operation", effs[0], typ))
    else:
        assert r == c["expect"]["value"]


def test_update_snapshot_and_nocreate():
    assert materializer.update_snapshot(TYPES["counter_pn"], 0, 1) == ("ok", 1)
    with pytest.raises(ValueError):
        materializer.create_snapshot("bla")


def test_corrupted_ops_cache_raises():
    typ = TYPES["counter_pn"]
    ops = [(2, ClocksiPayload("k", "antidote_crdt_set_aw", 1, {1: 1}, (1, 2), 2)),
           (1, ClocksiPayload("k", typ, 1, {1: 0}, (1, 1), 1))]
    with pytest.raises(CorruptedOpsCache):
        cm.materialize(typ, IGNORE, {1: 5}, SnapshotGetResponse(ops, 2, MaterializedSnapshot(0, 0)))


BEL = kats({"belongs_to_snapshot_op"})


def test_belongs_to_snapshot_kats():
    items = [(to_vc(c["sct"]), tuple(c["dc_ct"]), to_vc(c["op_ss"])) for c in BEL]
    got = materializer.belongs_to_snapshot_ops(items)
    assert got == [c["expect"]["result"] for c in BEL]
    assert materializer.belongs_to_snapshot_op(IGNORE, (1, 5), {1: 1}) is True


VNODE = kats({"vnode"})


@pytest.mark.parametrize("c", VNODE, ids=[c["name"] for c in VNODE])
def test_vnode_kat(c):
    typ = TYPES[c["type"]]
    v = MaterializerVnode()
    for st in c["steps"]:
        if st[0] == "update":
            v.update(st[1], payload(st[2], typ))
        else:
            _, key, r, gc, want = st
            ok, val = v.internal_read(key, typ, to_vc(r), IGNORE, gc)
            assert ok == "ok" and cm.value(typ, val) == want, st


def test_orddict_get_smaller_kats():
    for c in kats({"orddict_insert_then"}):
        d = VectorOrddict()
        for clock, val in c["inserts"]:
            d = d.insert(to_vc(clock), val)
        for chk in c["checks"]:
            if chk[0] != "get_smaller":
                continue
            found, first = d.get_smaller(to_vc(chk[1]))
            want = None if chk[2][0] is None else (to_vc(chk[2][0][0]), chk[2][0][1])
            assert (found, first) == (want, chk[2][1])


@pytest.mark.parametrize("c", kats({"gst"}), ids=[c["name"] for c in kats({"gst"})])
def test_gst_kat(c):
    parts = {p: ("undefined" if v == "undefined" else to_vc(v)) for p, v in c["parts"].items()}
    assert stable_time_functions.get_min_time(parts) == to_vc(c["expect"])


def test_update_stable_and_plugin():
    name, upd, merge, il, im = stable_time_functions.export_funcs_and_vals()
    assert name == "stable" and il == {} and im == {}
    assert upd(None, 3) and upd(3, 3) and not upd(4, 3)
    assert merge({"p1": {"dc1": 3}, "p2": {"dc1": 2}}) == {"dc1": 2}
    ch, acc = stable_time_functions.update_stable({"dc1": 5}, {"dc1": 7, "dc2": 1})
    assert ch and acc == {"dc1": 7, "dc2": 1}


@pytest.mark.parametrize("c", kats({"system_seq"}), ids=[c["name"] for c in kats({"system_seq"})])
def test_system_seq_kat(c):
    typ = TYPES[c["type"]]
    ops, reads, _ = system_seq_log(c)
    ops = [(i, ClocksiPayload(p.key, p.type, p.op_param, p.snapshot_time, p.commit_time, p.txid))
           for i, p in ops]
    exp = c["expect_after"]
    checks = (list(enumerate(exp)) if isinstance(exp, list)
              else [(int(k) - 1, v) for k, v in exp.items()])
    for i, want in checks:
        r = cm.materialize(typ, IGNORE, reads[i], SnapshotGetResponse(
            ops, len(ops), MaterializedSnapshot(0, cm.new(typ))))
        assert cm.value(typ, r[1]) == want
        if "expect_state_tokens_per_elem" in c:
            assert all(len(toks) == 1 for _, toks in r[1])


def test_vnode_all_pruned_keeps_zero_ops():
    """prune_ops with every op covered: the reference stores an empty tuple
    slot as the only op (:580-583), which its next materialize cannot read;
    the mirror (like the device GC, AGN_GC_ALL_PRUNED) keeps zero ops, sizes
    the list with NewLength = 1, and the key stays readable from its snapshot."""
    typ = "antidote_crdt_counter_pn"
    vn = MaterializerVnode()
    for i in range(1, 6):
        vn.update("k", ClocksiPayload("k", typ, i, {"dc1": 10 * i - 5}, ("dc1", 10 * i), i))
    assert vn.read("k", typ, {"dc1": 100}) == ("ok", 15)
    snaps = VectorOrddict()
    for t, v in ((60, 15), (70, 15), (80, 15)):
        snaps = snaps.insert_bigger({"dc1": t}, MaterializedSnapshot(5, v))
    vn.snapshot_insert_gc("k", snaps, True)
    t = vn.ops_cache["k"]
    assert t.length == 0 and t.list_len == 50 and t.op_counter == 5
    assert vn.read("k", typ, {"dc1": 100}) == ("ok", 15)
    vn.update("k", ClocksiPayload("k", typ, 7, {"dc1": 95}, ("dc1", 110), 6))
    assert vn.read("k", typ, {"dc1": 200}) == ("ok", 22)
