"""Multi-rank path of bench.py on CPU (gloo, world size 2).

The render shards by preset with no data-path collective:
each rank packs its own seeds, and only the timing barrier and the MAX
all-reduce of the elapsed time cross ranks.  These tests run that logic in two
gloo processes; the device render itself is covered by the -m gpu tests.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import bench


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, batch, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import msgpu
        from msgpu.pack import PackedBatch
        seeds = bench.rank_seeds(rank, batch)
        irs = bench.load_irs()
        packed = PackedBatch([msgpu.config_params("C2", seed=s, irs=irs) for s in seeds])
        elapsed = 0.25 * (rank + 1)            # rank 1 is the slow one
        dist.barrier()
        t = bench.max_over_ranks(elapsed, world, "cpu")
        q.put((rank, seeds, int(packed.total_frames), t))
    finally:
        dist.destroy_process_group()


def test_two_rank_sharding_gloo():
    world, batch = 2, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    seeds = [s for _, ss, _, _ in res for s in ss]
    assert seeds == list(range(1000, 1000 + world * batch))      # disjoint, contiguous
    assert all(t == pytest.approx(0.5) for *_, t in res)          # max over ranks
    assert res[0][2] == res[1][2] == batch * 192000               # C2: 1 s at 192 kHz


def test_single_rank_reduce_is_identity():
    assert bench.max_over_ranks(1.5, 1, "cpu") == 1.5
    assert np.array_equal(bench.rank_seeds(0, 4), [1000, 1001, 1002, 1003])
