"""The NIF's C (nif/antidote_gpu_nif.c) runs on the CPU through the minimal
erl_nif runtime (tests/nif_rt): load, the term runtime's codec, argument
checking (enif_make_badarg) and the error tuple of an engine call without a
device ({error, enodev}).  The GPU half is tests/test_nif_exec.py."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "nif_rt"))
import terms  # noqa: E402
from terms import Atom, NifBadarg  # noqa: E402


@pytest.fixture(scope="module")
def rt():
    terms.build()
    return terms.NifRuntime()


def test_codec_roundtrip(rt):
    for v in [0, -1, 2 ** 63, -(2 ** 63), 2 ** 64 - 1, Atom("ok"), (), (1, Atom("a"), [b"x"]),
              [], [1, [2, [3]], (4,)], b"", bytes(range(256)), [(Atom("dc1"), 17)] * 50]:
        assert terms.roundtrip(rt, v) == v, v


def test_open_without_device_is_an_error_tuple(rt):
    r = rt.call("open", 0)
    # no GPU in this container: agn_open -> AGN_ENODEV -> {error, enodev}
    # (on a GPU box the same call returns {ok, Ctx}; see test_nif_exec.py)
    assert r[0] in (Atom("error"), Atom("ok"))
    if r[0] == Atom("error"):
        assert r == (Atom("error"), Atom("enodev"))


@pytest.mark.parametrize("name,args", [
    ("open", (Atom("zero"),)),
    ("part_open", (Atom("not_a_ctx"), Atom("antidote_crdt_counter_pn"), 3, 10, True)),
    ("part_update", (Atom("nope"), 1, 1, [], Atom("ignore"), 5)),
    ("part_read", (Atom("nope"), 1, 1, [], Atom("ignore"), False)),
    ("materialize", (Atom("nope"), 1, 3, (), (), b"")),
    ("gst_min", (Atom("nope"), 3, 1, b"", b"")),
])
def test_malformed_arguments_are_badarg(rt, name, args):
    with pytest.raises(NifBadarg):
        rt.call(name, *args)


def test_unknown_function(rt):
    with pytest.raises(AttributeError):
        rt.call("no_such_nif", 1)
