"""World-size-2 CPU tests (torch.distributed gloo on 127.0.0.1) of the N>1
paths: vnode-partition sharding of the materialize batch and the GST
local-min -> MIN-allreduce -> finalize exchange.  The kernels are replaced by
the C oracle (CPU); what is tested is the placement and the exchange: each
rank's local vector (oracle_gst_min = agn_gst_min's contract) crosses ranks
through torch.distributed and is merged by the product's host exchange
agn_gst_merge (the all-gather + min of meta_data_sender, the transport-
agnostic twin of agn_gst_allreduce's RCCL min), with undefined partitions on
one rank so the flag word crosses ranks."""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle():
    from antidote_amd import _abi
    return _abi.bind(C.CDLL(os.path.join(ROOT, "oracle", "liboracle.so")), _abi.ORACLE_PROTOTYPES)


def _materialize_counts(cfg):
    from antidote_amd.encode import alloc_result, result_struct
    from antidote_amd.engine import free_gen_host, gen_host
    lib = _oracle()
    hl, hr = gen_host(cfg)
    r = alloc_result(cfg.n_keys, cfg.n_dcs, sparse=False)
    assert lib.oracle_materialize(C.byref(hl), C.byref(hr), C.byref(result_struct(r)), 1) == 0
    free_gen_host(hl, hr)
    return r


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from antidote_amd import _abi, sharding
        # ---- sharded materialize: rank r owns keys r + world*i
        base, stride = sharding.rank_key_stream(rank, world)
        n_local = 500
        cfg = _abi.AgnGenCfg(crdt_type=1, n_dcs=8, n_keys=n_local, ops_per_key=64, n_elems=0,
                             seed=20250113, key_base=base, key_stride=stride)
        r = _materialize_counts(cfg)
        for i in range(0, n_local, 97):  # every owned key maps to this rank
            assert sharding.rank_of_key(base + i * stride, world) == rank
        vals = torch.tensor(r.value.astype(np.int64))
        gathered = [torch.zeros_like(vals) for _ in range(world)]
        dist.all_gather(gathered, vals)
        # ---- GST: each rank owns partitions p with p % world == rank
        D, P = 6, 64
        lib = _abi.bind(C.CDLL(os.path.join(ROOT, "antidote_amd", "libantidote_gpu.so")),
                        _abi.PROTOTYPES)
        gsts = []
        for case, p_undef in enumerate((0.0, 0.05)):
            rng = np.random.default_rng(11 + case)
            clocks = (1_000_000 + rng.integers(0, 10 ** 6, (P, D))).astype(np.uint64)
            clocks[rng.random((P, D)) < 0.1] = np.uint64(sharding.U64_MAX)
            defined = (rng.random(P) >= p_undef).astype(np.uint8)
            if p_undef:   # undefined partitions on rank 1's side only
                defined[[p for p in range(P) if sharding.gpu_of(p, world) == 0]] = 1
                defined[1] = 0
            mine = [p for p in range(P) if sharding.gpu_of(p, world) == rank]
            local = np.zeros(D + 1, np.uint64)
            cm, dm = np.ascontiguousarray(clocks[mine]), np.ascontiguousarray(defined[mine])
            _oracle().oracle_gst_min(D, len(mine), 1, cm.ctypes.data, dm.ctypes.data,
                                     local.ctypes.data, 0)
            # the local vector is agn_gst_min's (before finalize): check it
            assert np.array_equal(local, sharding.local_gst_vector(cm, dm))
            vecs = [torch.zeros(D + 1, dtype=torch.int64) for _ in range(world)]
            dist.all_gather(vecs, torch.from_numpy(local.view(np.int64).copy()))
            allv = np.ascontiguousarray(np.stack([v.numpy() for v in vecs]).view(np.uint64))
            out = np.zeros(D + 1, np.uint64)
            assert lib.agn_gst_merge(D, world, allv.ctypes.data, out.ctypes.data) == 0
            gsts.append((out, clocks, defined))
        q.put((rank, [g.numpy() for g in gathered], gsts))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_world2_sharding_and_gst():
    from antidote_amd import _abi
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    outs.sort(key=lambda x: x[0])
    # sharded results == one rank materializing every global key
    full = _materialize_counts(_abi.AgnGenCfg(crdt_type=1, n_dcs=8, n_keys=1000, ops_per_key=64,
                                              n_elems=0, seed=20250113, key_base=0,
                                              key_stride=1))
    gathered = outs[0][1]
    for r in range(world):
        assert np.array_equal(gathered[r], full.value[r::world])
    # GST after the exchange == get_min_time over every partition (oracle)
    for case, (gst, clocks, defined) in enumerate(outs[0][2]):
        assert np.array_equal(outs[1][2][case][0], gst)
        want = np.zeros(clocks.shape[1] + 1, np.uint64)
        _oracle().oracle_gst_min(clocks.shape[1], clocks.shape[0], 1, clocks.ctypes.data,
                                 defined.ctypes.data, want.ctypes.data, 1)
        assert np.array_equal(gst, want)
        assert bool(want[-1] == 0) == bool((defined == 0).any())
