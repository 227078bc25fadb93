"""Multi-GPU sharding of independent frame pairs, rehearsed on CPU with gloo (world size 2).

Each rank takes its contiguous block of pairs (svo_amd.shard.pair_block), aligns it (here with the CPU
oracle, since this container has no GPU; on the GPU box bench.py runs the HIP path per rank), and the
blocks are gathered in rank order.  The gathered poses must equal the single-process result bit for bit:
pairs share nothing, so the result cannot depend on the GPU count.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import svo_amd.shard as shard
import svo_amd.synth as synth

N_PAIRS, NF, LEVELS = 5, 120, 3


def test_pair_block_partition():
    for n in (0, 1, 5, 8, 512, 513):
        for world in (1, 2, 3, 8):
            blocks = [shard.pair_block(n, r, world) for r in range(world)]
            assert sum(c for _, c in blocks) == n
            nxt = 0
            for r, (first, count) in enumerate(blocks):
                assert first == nxt
                for p in range(first, first + count):
                    assert shard.owner(p, n, world) == r
                nxt = first + count
    assert shard.pair_block(512, 3, 8) == (192, 64)  # config 4: 64 pairs per GPU
    with pytest.raises(ValueError):
        shard.pair_block(4, 2, 2)


def _align_block(first, count):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "tests"))
    from common import oracle_align
    out = []
    for i in range(first, first + count):
        s = synth.make_pair(seed=synth.SEED_BASE + i, n_features=NF, nthreads=1)
        pose, err, st, _ = oracle_align(s, 5, 0, LEVELS - 1, mode=0, trace=False)
        out.append((pose.tolist(), float(err), int(st)))
    return out


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        first, count = shard.pair_block(N_PAIRS, rank, world)
        res = shard.gather_blocks(_align_block(first, count), dist)
        if rank == 0:
            q.put(res)
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_gloo_gather_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world = 2
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _align_block(0, N_PAIRS)
    assert len(got) == N_PAIRS
    for (pg, eg, sg), (pr, er, sr) in zip(got, ref):
        assert np.array_equal(np.array(pg), np.array(pr)) and (eg == er or (np.isnan(eg) and np.isnan(er))) and sg == sr
