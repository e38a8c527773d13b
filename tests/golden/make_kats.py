"""Write tests/golden/kats.json: the reference's hot-path known-answer tests.

Each case is a hand transcription of one EUnit / common_test assertion of the
AntidoteDB reference (paths relative to its tree).  Only values the reference
ASSERTS are recorded under "expect"; the reference cannot run here (no Erlang
runtime), so these fixtures are the pin for both oracles.

Encoding: a vector clock is a list of [dc, time] pairs; a DC id is the Erlang
term written as a JSON int or string; a payload is
{"p": op_param, "ss": clock, "ct": [dc, time], "tx": txid}.

Run:  python tests/golden/make_kats.py   (rewrites kats.json)
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def vc(*pairs):
    return [list(p) for p in pairs]


def pl(p, ct, ss, tx):
    return {"p": p, "ct": list(ct), "ss": vc(*ss), "tx": tx}


CASES = []


def add(**kw):
    CASES.append(kw)


# --------------------------------------------------------------------------
# src/clocksi_materializer.erl
# materializer_clocksi_test :279-313
ops = [[4, pl(2, (1, 4), [(1, 4)], 4)], [3, pl(1, (1, 3), [(1, 3)], 3)],
       [2, pl(1, (1, 2), [(1, 2)], 2)], [1, pl(2, (1, 1), [(1, 1)], 1)]]
for r, val, hole, ct in [((1, 3), 4, 3, [(1, 3)]), ((1, 4), 6, 4, [(1, 4)]),
                         ((1, 7), 6, 4, [(1, 4)])]:
    add(kind="materialize", name=f"materializer_clocksi_test R={r}",
        src="src/clocksi_materializer.erl:279-313", type="counter_pn",
        txid=None, R=vc(r), sct=None, base=[0, 0], ops=ops,
        expect={"value": val, "hole": hole, "ct": vc(*ct)})

# materializer_missing_op_test :319-349
ops = [[4, pl(1, (1, 3), [(1, 2), (2, 1)], 2)], [3, pl(1, (2, 2), [(1, 1), (2, 1)], 3)],
       [2, pl(1, (1, 2), [(1, 2), (2, 1)], 2)], [1, pl(1, (1, 1), [(1, 1), (2, 1)], 1)]]
add(kind="materialize", name="materializer_missing_op_test step1",
    src="src/clocksi_materializer.erl:339-342", type="counter_pn", txid=None,
    R=vc((1, 3), (2, 1)), sct=None, base=[0, 0], ops=ops,
    expect={"value": 3, "ct": vc((1, 3), (2, 1))})
add(kind="materialize_chain", name="materializer_missing_op_test step2",
    src="src/clocksi_materializer.erl:344-349", type="counter_pn", txid=None,
    first={"R": vc((1, 3), (2, 1)), "sct": None, "base": [0, 0]},
    R=vc((1, 3), (2, 2)), ops=ops,
    expect={"value": 4, "hole": 4, "ct": vc((1, 3), (2, 2))})

# materializer_missing_dc_test :354-396 (sparse clocks)
ops = [[4, pl(1, (1, 3), [(1, 2)], 2)], [3, pl(1, (2, 2), [(2, 1)], 3)],
       [2, pl(1, (1, 2), [(1, 2)], 2)], [1, pl(1, (1, 1), [(1, 1)], 1)]]
add(kind="materialize", name="materializer_missing_dc_test A",
    src="src/clocksi_materializer.erl:374-377", type="counter_pn", txid=None,
    R=vc((1, 3)), sct=None, base=[0, 0], ops=ops,
    expect={"value": 3, "ct": vc((1, 3))})
add(kind="materialize_chain", name="materializer_missing_dc_test B",
    src="src/clocksi_materializer.erl:379-384", type="counter_pn", txid=None,
    first={"R": vc((1, 3)), "sct": None, "base": [0, 0]},
    R=vc((1, 3), (2, 2)), ops=ops,
    expect={"value": 4, "hole": 4, "ct": vc((1, 3), (2, 2))})
add(kind="materialize", name="materializer_missing_dc_test C",
    src="src/clocksi_materializer.erl:386-389", type="counter_pn", txid=None,
    R=vc((1, 3), (2, 1)), sct=None, base=[0, 0], ops=ops,
    expect={"value": 3, "ct": vc((1, 3))})
add(kind="materialize_chain", name="materializer_missing_dc_test D",
    src="src/clocksi_materializer.erl:391-396", type="counter_pn", txid=None,
    first={"R": vc((1, 3), (2, 1)), "sct": None, "base": [0, 0]},
    R=vc((1, 3), (2, 2)), ops=ops,
    expect={"value": 4, "hole": 4, "ct": vc((1, 3), (2, 2))})

# materializer_clocksi_concurrent_test :398-430
ops = [[3, pl(1, (1, 2), [(1, 2), (2, 1)], 2)], [2, pl(1, (2, 2), [(1, 1), (2, 1)], 3)],
       [1, pl(2, (1, 1), [(1, 1), (2, 1)], 1)]]
for r, val, hole, ct, src in [
        (vc((2, 2), (1, 2)), 4, 3, vc((1, 2), (2, 2)), ":413-418"),
        (vc((1, 2), (2, 1)), 3, 1, vc((1, 2), (2, 1)), ":422-424"),
        (vc((1, 1), (2, 2)), 3, 2, vc((1, 1), (2, 2)), ":425-427"),
        (vc((1, 1), (2, 1)), 2, 1, vc((1, 1), (2, 1)), ":428-430")]:
    add(kind="materialize", name=f"materializer_clocksi_concurrent_test R={r}",
        src="src/clocksi_materializer.erl" + src, type="counter_pn", txid=None,
        R=r, sct=None, base=[0, 0], ops=ops,
        expect={"value": val, "hole": hole, "ct": ct})

# materializer_clocksi_noop_test :433-442
add(kind="materialize", name="materializer_clocksi_noop_test",
    src="src/clocksi_materializer.erl:433-442", type="counter_pn", txid=None,
    R=vc((1, 1)), sct=None, base=[0, 0], ops=[],
    expect={"value": 0, "hole": 0, "ct": None})

# materializer_eager_clocksi_test :444-458 and materializer.erl eager tests
for effs, val, name, src in [
        ([], 0, "materializer_eager_clocksi_test (no ops)", "src/clocksi_materializer.erl:448-450"),
        ([1, 2, 3, 4], 10, "materializer_eager_clocksi_test", "src/clocksi_materializer.erl:452-458"),
        ([1], 1, "update_pncounter_test", "src/materializer.erl:112-118"),
        ([1, 1, 2, 3], 7, "materializer_counter_withlog_test", "src/materializer.erl:121-131"),
        ([], 0, "materializer_counter_emptylog_test", "src/materializer.erl:134-140")]:
    add(kind="eager", name=name, src=src, type="counter_pn", effects=effs,
        expect={"value": val})
add(kind="eager", name="materializer_error_invalidupdate_test",
    src="src/materializer.erl:147-155", type="counter_pn",
    effects=[{"invalid": "{non_existing_op_type, {non_existing_op, actor1}}"}],
    expect={"error": "unexpected_operation", "op_index": 0})

# is_op_in_snapshot_test :460-470
add(kind="is_op_in_snapshot", name="is_op_in_snapshot_test ST1",
    src="src/clocksi_materializer.erl:469", txid=2,
    op=pl(["increment", 2], ("dc1", 1), [("dc1", 1)], 1), snapshot=vc(("dc1", 2)),
    expect={"incl": True, "in_prev": False, "time": vc(("dc1", 1))})
add(kind="is_op_in_snapshot", name="is_op_in_snapshot_test ST2",
    src="src/clocksi_materializer.erl:470", txid=2,
    op=pl(["increment", 2], ("dc1", 1), [("dc1", 1)], 1), snapshot=vc(("dc1", 0)),
    expect={"incl": False, "in_prev": False, "time": None})

# src/materializer.erl belongs_to_snapshot_test :173-193
snap = vc((1, 5), (2, 5))
for sct, dcct, want in [(vc((1, 1), (2, 1)), (1, 5), True), (vc((1, 1), (2, 7)), (2, 5), True),
                        (vc((1, 5), (2, 10)), (1, 5), False), (vc((1, 5), (2, 10)), (2, 5), False)]:
    add(kind="belongs_to_snapshot_op", name=f"belongs_to_snapshot_test {sct} {dcct}",
        src="src/materializer.erl:186-193", sct=sct, dc_ct=list(dcct), op_ss=snap,
        expect={"result": want})


# --------------------------------------------------------------------------
# src/materializer_vnode.erl (counter_pn; effect of downstream({increment,1}) = 1)
def upd(key, ss, ct, tx=1):
    return ["update", key, {"p": 1, "ss": vc(*ss), "ct": list(ct), "tx": tx}]


def rd(key, r, gc, want):
    return ["read", key, vc(*r), gc, want]


steps = []
for n in range(0, 11):
    steps.append(rd("mycount", [(1, n * 10 + 2)], False, n))
    steps.append(upd("mycount", [(1, n * 10)], (1, n * 10 + 1)))
steps += [upd("mycount", [(1, 15)], (1, 111)), upd("mycount", [(1, 16)], (1, 121)),
          rd("mycount", [(1, 102)], True, 11), upd("mycount", [(1, 102)], (1, 131)),
          rd("mycount", [(1, 142)], True, 14)]
add(kind="vnode", name="gc_test", src="src/materializer_vnode.erl:652-682",
    type="counter_pn", steps=steps)

steps = [rd("mycount", [(1, 2)], False, 0)]
steps += [upd("mycount", [(1, 10)], (1, 11 + v)) for v in range(1, 1001)]
steps.append(rd("mycount", [(1, 2000)], False, 1000))
for v in range(1001, 1101):
    steps.append(upd("mycount", [(1, 10 + v)], (1, 11 + v)))
    steps.append(rd("mycount", [(1, 2000)], False, v))
add(kind="vnode", name="large_list_test", src="src/materializer_vnode.erl:685-709",
    type="counter_pn", steps=steps)

add(kind="vnode", name="seq_write_test", src="src/materializer_vnode.erl:724-759",
    type="counter_pn", steps=[
        upd("mycount", [(1, 10)], (1, 15), 1), rd("mycount", [(1, 16)], False, 1),
        upd("mycount", [(1, 16)], (1, 20), 2), rd("mycount", [(1, 21)], False, 2),
        rd("mycount", [(1, 16)], False, 1)])
add(kind="vnode", name="multipledc_write_test", src="src/materializer_vnode.erl:761-798",
    type="counter_pn", steps=[
        upd("mycount", [(2, 0), (1, 10)], (1, 15), 1),
        rd("mycount", [(1, 16), (2, 0)], False, 1),
        upd("mycount", [(2, 16), (1, 16)], (2, 20), 2),
        rd("mycount", [(1, 16), (2, 21)], False, 2),
        rd("mycount", [(1, 15), (2, 15)], False, 1)])
add(kind="vnode", name="concurrent_write_test", src="src/materializer_vnode.erl:800-842",
    type="counter_pn", steps=[
        upd("mycount", [("local", 0), ("remote", 0)], ("remote", 1), 1),
        rd("mycount", [("remote", 1), ("local", 0)], False, 1),
        upd("mycount", [("local", 0), ("remote", 0)], ("local", 1), 2),
        rd("mycount", [("local", 1), ("remote", 0)], False, 1),
        rd("mycount", [("local", 0), ("remote", 1)], False, 1),
        rd("mycount", [("remote", 1), ("local", 1)], False, 2)])
add(kind="vnode", name="read_nonexisting_key_test", src="src/materializer_vnode.erl:846-852",
    type="counter_pn", steps=[rd("key", [("dc1", 1), ("dc2", 0)], False, 0)])


# --------------------------------------------------------------------------
# src/vector_orddict.erl :187-267
CT1, CT2, CT3 = vc(("dc1", 4), ("dc2", 4)), vc(("dc1", 8), ("dc2", 8)), vc(("dc1", 1), ("dc2", 10))
add(kind="orddict_insert_then", name="vector_oddict_get_smaller_from_id_test",
    src="src/vector_orddict.erl:187-201", inserts=[[CT1, 1], [CT2, 2], [CT3, 3]],
    checks=[["get_smaller_from_id", ["dc1", 0], None, "empty"],
            ["get_smaller_from_id", ["dc1", 0], None],
            ["get_smaller_from_id", ["dc1", 1], [CT3, 3]],
            ["get_smaller_from_id", ["dc2", 9], [CT2, 2]]])
add(kind="orddict_insert_then", name="vector_orddict_get_smaller_test",
    src="src/vector_orddict.erl:204-219", inserts=[[CT1, 1], [CT2, 2], [CT3, 3]],
    checks=[["get_smaller", vc(("dc1", 0), ("dc2", 0)), [None, False]],
            ["get_smaller", vc(("dc1", 1), ("dc2", 6)), [None, False]],
            ["get_smaller", vc(("dc1", 5), ("dc2", 5)), [[CT1, 1], False]],
            ["get_smaller", vc(("dc1", 9), ("dc2", 9)), [[CT2, 2], True]],
            ["get_smaller", vc(("dc1", 3), ("dc2", 11)), [[CT3, 3], False]]])
add(kind="orddict_insert_bigger", name="vector_orddict_insert_bigger_test",
    src="src/vector_orddict.erl:223-236",
    steps=[[vc(("dc1", 4), ("dc2", 4)), 1, 1], [vc(("dc1", 3), ("dc2", 3)), 2, 1],
           [vc(("dc1", 6), ("dc2", 10)), 3, 2]])
three = [[vc(("dc1", 4), ("dc2", 4)), "snapshot_1"], [vc(("dc1", 0), ("dc2", 3)), "snapshot_2"],
         [vc(), "snapshot_3"]]
add(kind="orddict_filter_gt_new", name="vector_orddict_filter_test",
    src="src/vector_orddict.erl:238-255", entries=three,
    expect=[three[0], three[1]])
add(kind="orddict_conc", name="vector_orddict_conc_test",
    src="src/vector_orddict.erl:257-267", entries=three,
    checks=[[vc(("dc1", 3), ("dc2", 3)), False], [vc(("dc1", 2), ("dc2", 1)), True]])


# --------------------------------------------------------------------------
# src/meta_data_sender.erl GST tests :384-490 (the get_min_time merge each
# asserts; partition bookkeeping via the ring is out of scope)
U = "undefined"
for name, src, parts, want in [
        ("merge_test 1", ":394-398", {"p1": vc(("dc1", 10), ("dc2", 5)), "p2": vc(("dc1", 5), ("dc2", 10))},
         vc(("dc1", 5), ("dc2", 5))),
        ("merge_test 2", ":400-407", {"p1": vc(("dc1", 10), ("dc2", 5)), "p2": vc(("dc1", 5), ("dc2", 10)),
                                      "p3": vc(("dc1", 20), ("dc2", 20))}, vc(("dc1", 5), ("dc2", 5))),
        ("empty_test", ":418-424", {"p1": vc(), "p2": vc(), "p3": vc()}, vc()),
        ("missing_test", ":433-441", {"p1": vc(("dc1", 10)), "p2": U, "p3": vc(("dc1", 10))},
         vc(("dc1", 0))),
        ("merge_node_change_test 1", ":454-459", {"p1": vc(("dc1", 10), ("dc2", 5)),
                                                  "p2": vc(("dc1", 5), ("dc2", 10))},
         vc(("dc1", 5), ("dc2", 5))),
        ("merge_node_change_test 2", ":461-468", {"p1": vc(("dc1", 10), ("dc2", 10)),
                                                  "p3": vc(("dc1", 20), ("dc2", 20))},
         vc(("dc1", 10), ("dc2", 10))),
        ("merge_node_delete_test 1", ":478-485", {"p3": vc(("dc1", 0), ("dc2", 0)),
                                                  "p1": vc(("dc1", 10), ("dc2", 5)),
                                                  "p2": vc(("dc1", 5), ("dc2", 10))},
         vc(("dc1", 0), ("dc2", 0))),
        ("merge_node_delete_test 2", ":487-490", {"p1": vc(("dc1", 10), ("dc2", 5)),
                                                  "p2": vc(("dc1", 5), ("dc2", 10))},
         vc(("dc1", 5), ("dc2", 5)))]:
    add(kind="gst", name=name, src="src/meta_data_sender.erl" + src, parts=parts, expect=want)


# --------------------------------------------------------------------------
# System tests (common_test; not runnable here) — sequential single-DC logs.
# set_aw add a, add b, remove a: test/singledc/clocksi_SUITE.erl:160-180
add(kind="system_seq", name="clocksi_test5 set_aw", src="test/singledc/clocksi_SUITE.erl:160-180",
    type="set_aw", updates=[["add", "a"], ["add", "b"], ["remove", "a"]],
    expect_after=[["a"], ["a", "b"], ["b"]])
# register_mv assign a, b, c: test/singledc/clocksi_SUITE.erl:184-206
add(kind="system_seq", name="clocksi_multiple_updates_per_txn_test register_mv",
    src="test/singledc/clocksi_SUITE.erl:184-206", type="register_mv",
    updates=[["assign", "a"], ["assign", "b"], ["assign", "c"]],
    expect_after=[["a"], ["b"], ["c"]])
# set_aw state layout: one token per element after 15 adds, then 30 elements
add(kind="system_seq", name="object_log_state_test", src="test/singledc/object_log_state_SUITE.erl:63-109",
    type="set_aw", updates=[["add", i] for i in range(1, 31)],
    expect_after={"15": list(range(1, 16)), "30": list(range(1, 31))},
    expect_state_tokens_per_elem=1)


# --------------------------------------------------------------------------
# System tests with a multi-DC / multi-key / multi-update transaction history
# (kind "system_txn"; tests/kat_util.py system_txn_log gives the clock model).
# A txn is {"dc", "dep": [txn indices] (the causal dependency clock passed to
# update_*: the max of their commit times; [] = ignore), "updates", "key"}; a
# read is {"key", "at": [txn indices] (read clock = max of their commit
# times), "expect": the value the reference asserts}.
def tx(dc, updates, dep=(), key="k"):
    return {"dc": dc, "dep": list(dep), "updates": updates, "key": key}


def rd_at(at, expect, key="k"):
    return {"key": key, "at": list(at), "expect": expect}


INC = [["increment", 1]]

# inter_dc_repl_SUITE causality_test: add first, add second in DC1, remove
# first in DC2 (each depending on the previous commit) -> [second]
add(kind="system_txn", name="inter_dc_repl causality_test set_aw",
    src="test/multidc/inter_dc_repl_SUITE.erl:122-139", type="set_aw",
    txns=[tx("dc1", [["add", "first"]]), tx("dc1", [["add", "second"]], [0]),
          tx("dc2", [["remove", "first"]], [1])],
    reads=[rd_at([2], ["second"])])
# inter_dc_repl_SUITE simple_replication_test: 3 increments in DC1, read on DC1
# and DC2 at the last commit time -> 3
add(kind="system_txn", name="inter_dc_repl simple_replication_test",
    src="test/multidc/inter_dc_repl_SUITE.erl:87-100", type="counter_pn",
    txns=[tx("dc1", INC) for _ in range(3)], reads=[rd_at([2], 3)])
# inter_dc_repl_SUITE multiple_keys_test: 10 rounds of one increment on each of
# 10 keys, one more increment on the base key; every derived key reads 10
txns = [tx("dc1", INC, key=f"mk{n}") for _ in range(10) for n in range(1, 11)]
txns.append(tx("dc1", INC, key="multiple_keys_test"))
add(kind="system_txn", name="inter_dc_repl multiple_keys_test",
    src="test/multidc/inter_dc_repl_SUITE.erl:103-118,187-206", type="counter_pn",
    txns=txns, reads=[rd_at([len(txns) - 1], 10, key=f"mk{n}") for n in range(1, 11)])
# multiple_dcs_SUITE simple_replication_test: 3 in DC1 -> 3; +1 in DC2 after
# CommitTime, +1 in DC3 after CommitTime2 -> 5 on every DC
add(kind="system_txn", name="multiple_dcs simple_replication_test",
    src="test/multidc/multiple_dcs_SUITE.erl:89-117", type="counter_pn",
    txns=[tx("dc1", INC), tx("dc1", INC), tx("dc1", INC), tx("dc2", INC, [2]),
          tx("dc3", INC, [3])],
    reads=[rd_at([2], 3), rd_at([4], 5)])
# multiple_dcs_SUITE parallel_writes_test: 5 increments on each of 3 DCs
# concurrently (no dependency), read at the merged max of the 3 commit times -> 15
txns = [tx(f"dc{d}", INC) for _ in range(5) for d in (1, 2, 3)]
add(kind="system_txn", name="multiple_dcs parallel_writes_test",
    src="test/multidc/multiple_dcs_SUITE.erl:120-165", type="counter_pn",
    txns=txns, reads=[rd_at([12, 13, 14], 15)])
# multiple_dcs_SUITE blocking_test: +1 in DC1, +1 in DC2, read at
# vectorclock:max of both commit times -> 2
add(kind="system_txn", name="multiple_dcs blocking_test",
    src="test/multidc/multiple_dcs_SUITE.erl:212-240", type="counter_pn",
    txns=[tx("dc1", INC), tx("dc2", INC)], reads=[rd_at([0, 1], 2)])
# multiple_dcs_SUITE replicated_set_test: 100 adds on DC1 -> lists:seq(1, 100)
# (more than one 64-entry chunk of the tag kernel)
add(kind="system_txn", name="multiple_dcs replicated_set_test",
    src="test/multidc/multiple_dcs_SUITE.erl:243-266", type="set_aw",
    txns=[tx("dc1", [["add", n]]) for n in range(1, 101)],
    reads=[rd_at([99], list(range(1, 101)))])
# pb_client_SUITE (antidotec PB client; one single-DC transaction per commit)
add(kind="system_txn", name="pb_client pb_test_set_read_write",
    src="test/singledc/pb_client_SUITE.erl:186-202", type="set_aw",
    txns=[tx("dc1", [["add", "a"]])], reads=[rd_at([0], ["a"])])
add(kind="system_txn", name="pb_client update_set_read_test add_all",
    src="test/singledc/pb_client_SUITE.erl:259-282", type="set_aw",
    txns=[tx("dc1", [["add_all", ["a", "b"]]])], reads=[rd_at([0], ["a", "b"])])
add(kind="system_txn", name="pb_client static_transaction_test add_all",
    src="test/singledc/pb_client_SUITE.erl:491-517", type="set_aw",
    txns=[tx("dc1", [["add_all", ["a", "b"]]])], reads=[rd_at([0], ["a", "b"])])
add(kind="system_txn", name="pb_client crdt_mvreg_test",
    src="test/singledc/pb_client_SUITE.erl:305-321", type="register_mv",
    txns=[tx("dc1", [["assign", "a"]])], reads=[rd_at([0], ["a"])])
add(kind="system_txn", name="pb_client update_counter_crdt_and_read_test",
    src="test/singledc/pb_client_SUITE.erl:237-256", type="counter_pn",
    txns=[tx("dc1", [["increment", 15]])], reads=[rd_at([0], 15)])
# CRDTs embedded in the map tests: the map's entry value is the embedded
# CRDT's own value
add(kind="system_txn", name="pb_client crdt_gmap_test embedded set_aw add_all",
    src="test/singledc/pb_client_SUITE.erl:359,379", type="set_aw",
    txns=[tx("dc1", [["add_all", ["Apple", "Banana"]]])],
    reads=[rd_at([0], ["Apple", "Banana"])])
add(kind="system_txn", name="pb_client crdt_gmap_test embedded register_mv",
    src="test/singledc/pb_client_SUITE.erl:354,358,376,378", type="register_mv",
    txns=[tx("dc1", [["assign", "42"]], key="a"), tx("dc1", [["assign", "Paul"]], key="c")],
    reads=[rd_at([0], ["42"], key="a"), rd_at([1], ["Paul"], key="c")])
# crdt_map_rr_test: one transaction assigns b1..b5, then removes them through
# the map (map_rr remove = reset of the embedded register_mv); the asserted map
# holds no b1..b5 entry (map_rr hides bottom = empty registers), keeps b = [X]
# and i = [X], and d / e (set_aw add_all) = [Apple, Banana]
add(kind="system_txn", name="pb_client crdt_map_rr_test embedded register_mv reset",
    src="test/singledc/pb_client_SUITE.erl:401-458", type="register_mv",
    txns=[tx("dc1", [["assign", "X1"], ["reset", None]], key="b1"),
          tx("dc1", [["assign", "X4"], ["reset", None]], key="b4"),
          tx("dc1", [["assign", "X"]], key="b"), tx("dc1", [["assign", "X"]], key="i")],
    reads=[rd_at([0], [], key="b1"), rd_at([1], [], key="b4"), rd_at([2], ["X"], key="b"),
           rd_at([3], ["X"], key="i")])
add(kind="system_txn", name="pb_client crdt_map_rr_test embedded set_aw add_all",
    src="test/singledc/pb_client_SUITE.erl:413-414,452-453", type="set_aw",
    txns=[tx("dc1", [["add_all", ["Apple", "Banana"]]], key="d"),
          tx("dc1", [["add_all", ["Apple", "Banana"]]], key="e")],
    reads=[rd_at([0], ["Apple", "Banana"], key="d"), rd_at([1], ["Apple", "Banana"], key="e")])


if __name__ == "__main__":
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump({"reference": "anshulahuja98/antidote @ 2025-01-12", "cases": CASES}, f,
                  indent=1)
    print(f"wrote {len(CASES)} cases")
