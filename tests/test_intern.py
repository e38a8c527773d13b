"""agn_interner (host-only, no GPU): the exact term <-> integer maps of the
Erlang binding.  TxId equality must be exact (is_op_in_snapshot's
`TxId == Op#clocksi_payload.txid`, src/clocksi_materializer.erl:220): two
distinct terms never share an id, whatever their hashes."""
import threading

import numpy as np
import pytest

from antidote_amd._lib import EngineUnavailable
from antidote_amd.engine import Interner


def _interner(**kw):
    try:
        return Interner(**kw)
    except (EngineUnavailable, OSError) as e:  # pragma: no cover
        pytest.skip(f"library unavailable: {e}")


def test_exact_and_dense():
    with _interner(first_id=1) as t:
        terms = [b"", b"\x00", b"\x00\x00", b"a", b"ab", b"abc", b"b", bytes(range(256)),
                 b"\x83h\x03d\x00\x05tx_idb\x00\x00\x00\x01", b"\x83h\x03d\x00\x05tx_idb\x00\x00\x00\x02"]
        ids = [t.intern(x) for x in terms]
        assert [i for i, _ in ids] == list(range(1, len(terms) + 1))
        assert all(new for _, new in ids)
        again = [t.intern(x) for x in terms]
        assert [i for i, _ in again] == [i for i, _ in ids] and not any(n for _, n in again)
        for x, (i, _) in zip(terms, ids):
            assert t.bytes_of(i) == x and t.find(x) == i
        assert t.find(b"zzz") is None and len(t) == len(terms)
        with pytest.raises(Exception):
            t.bytes_of(0)
        with pytest.raises(Exception):
            t.bytes_of(len(terms) + 1)


def test_many_random_terms_no_sharing():
    rng = np.random.default_rng(5)
    with _interner(first_id=100) as t:
        seen = {}
        for _ in range(20000):
            n = int(rng.integers(0, 24))
            b = rng.integers(0, 4, n).astype(np.uint8).tobytes()   # many near-duplicates
            i, new = t.intern(b)
            assert new == (b not in seen)
            assert seen.setdefault(b, i) == i
        assert len(set(seen.values())) == len(seen) == len(t)
        assert min(seen.values()) == 100 and max(seen.values()) == 99 + len(seen)


def test_capacity():
    with _interner(first_id=0, max_ids=3) as t:
        for b in (b"x", b"y", b"z"):
            t.intern(b)
        assert t.intern(b"y") == (1, False)
        with pytest.raises(Exception, match="full"):
            t.intern(b"w")


def test_threads_agree():
    """16 threads intern overlapping term sets concurrently: one id per term."""
    words = [f"dc{i % 97}:{i // 97}".encode() for i in range(4000)]
    with _interner() as t:
        out = [dict() for _ in range(16)]

        def body(j):
            rng = np.random.default_rng(j)
            for w in rng.permutation(len(words)):
                out[j][words[w]] = t.intern(words[w])[0]
        ts = [threading.Thread(target=body, args=(j,)) for j in range(16)]
        for x in ts:
            x.start()
        for x in ts:
            x.join()
        for j in range(1, 16):
            assert out[j] == out[0]
        assert sorted(out[0].values()) == list(range(1, len(words) + 1))
