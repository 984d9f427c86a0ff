"""Multi-rank sharding path on CPU (gloo, world size 2 and 3): block partition,
uneven all-gather of per-rank results, max-over-ranks timing — the pieces
bench.py and the sharded rollout use over RCCL on the GPU node."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from nbody_amd.parallel import shard_range


def test_shard_range_partitions():
    for total in (0, 1, 7, 1024, 4097):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, r, world) for r in range(world)]
            assert sum(c for _, c in spans) == total
            pos = 0
            for s, c in spans:
                assert s == pos
                pos += c
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from nbody_amd import parallel as P
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        start, count = P.shard_range(total, rank, world)
        # each rank "simulates" its own systems: value = global system id
        local = torch.arange(start, start + count, dtype=torch.float64)[:, None, None].repeat(1, 4, 3)
        full = P.all_gather_shards(local, total)
        t = P.max_over_ranks(0.5 + rank)
        P.barrier()
        q.put((rank, full.shape, bool(torch.equal(full[:, 0, 0], torch.arange(total, dtype=torch.float64))), t))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,total", [(2, 1024), (2, 5), (3, 10)])
def test_gather_and_timing_over_gloo(world, total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, shape, ok, t in res:
        assert shape == (total, 4, 3) and ok
        assert t == 0.5 + world - 1
