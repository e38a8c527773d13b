"""Key → partition → GPU placement and the GST exchange algebra.

Placement restates log_utilities:get_key_partition for integer keys
(`Pos = Key rem NumPartitions + 1`, src/log_utilities.erl:65-70): partition
p = |key| mod P (P = 64, the riak_core default ring), GPU g = p mod G.  For
G | P the keys of rank r are exactly {r + G*i}: the generator's
(key_base = r, key_stride = G) streams, and materialize needs no exchange.

GST exchange (src/meta_data_sender.erl:230-255): each rank reduces its own
partitions to a vector of D+1 words (per-DC min, absent = UINT64_MAX; word D =
1 iff every partition was defined); the element-wise MIN of those vectors over
ranks is the global merge (RCCL ncclMin on ncclUint64 in agn_gst_allreduce);
the undefined => 0 rule is applied once, after the exchange.
"""
from __future__ import annotations

import numpy as np

RING_SIZE = 64
U64_MAX = (1 << 64) - 1


def partition_of(key: int, n_partitions: int = RING_SIZE) -> int:
    return abs(int(key)) % n_partitions


def gpu_of(partition: int, n_gpus: int) -> int:
    return partition % n_gpus


def rank_of_key(key: int, n_gpus: int, n_partitions: int = RING_SIZE) -> int:
    return gpu_of(partition_of(key, n_partitions), n_gpus)


def rank_key_stream(rank: int, world: int, n_partitions: int = RING_SIZE):
    """(key_base, key_stride) of the keys a rank owns; needs world | P."""
    if n_partitions % world:
        raise ValueError(f"{world} GPUs do not divide the {n_partitions}-partition ring")
    return rank, world


def local_gst_vector(clocks: np.ndarray, defined: np.ndarray | None) -> np.ndarray:
    """[P][D] u64 (absent = U64_MAX) -> [D+1] (what agn_gst_min computes)."""
    P, D = clocks.shape
    out = np.full(D + 1, U64_MAX, np.uint64)
    out[D] = 1
    for p in range(P):
        if defined is not None and not defined[p]:
            out[D] = 0
            continue
        out[:D] = np.minimum(out[:D], clocks[p])
    return out


def merge_vectors(vecs) -> np.ndarray:
    """The allreduce: element-wise min, flag word included."""
    out = np.array(vecs[0], np.uint64)
    for v in vecs[1:]:
        out = np.minimum(out, np.asarray(v, np.uint64))
    return out


def finalize(vec: np.ndarray) -> np.ndarray:
    D = len(vec) - 1
    out = np.array(vec, np.uint64)
    if out[D] == 0:
        out[:D][out[:D] != np.uint64(U64_MAX)] = 0
    return out
