"""CPU half of tests/test_ss_states.py: the keys its batcher comparison would
leave out (the reference's all-pruned placeholder and badmatch paths,
DESIGN.md §9) are computed from the reference transcription alone, for every
parametrization -- and there are none, so the GPU test compares every key
and asserts its exclusion set is empty."""
import pytest

from antidote_amd import _abi
import test_ss_states as t

CASES = sorted({(d, lg) for d, lg, _ in t.BATCHER_CASES})


@pytest.mark.parametrize("typ", [_abi.SET_AW, _abi.REGISTER_MV])
def test_reference_excludes_no_key(typ):
    for d, lg in CASES:
        assert t.reference_quirks(typ, d, lg) == set(), (typ, d, lg)
