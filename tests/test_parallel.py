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


# ------------------------------------------------------------------ SyncBN + sharded rollout
def _bn_sums(m, M):
    """[3][M] sums the producing kernels accumulate (tp_fused.h BnSrc): sum s, sum s^2 over
    the 0e channels, sum |v|^2 over the 1o channels, for m [rows, M + 3M] (e3nn layout)."""
    s = m[:, :M]
    v = m[:, M:].reshape(-1, M, 3)
    return torch.cat([s.sum(0), (s * s).sum(0), (v * v).sum(2).sum(0)])


def _syncbn_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import ctypes

    import numpy as np
    import torch.distributed as dist

    from nbody_amd.segnn import SEGNN
    from oracle.e3nn_lite import Irreps, batch_norm
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        M = 8
        rng = np.random.default_rng(0)
        full = rng.standard_normal((40, 4 * M)) * 1.5 + 0.3          # 40 message rows, 8x0e + 8x1o
        start, count = rank * 40 // world, (rank + 1) * 40 // world - rank * 40 // world
        part = torch.tensor(full[start:start + count])
        model = SEGNN(hidden_features=16, num_layers=1).enable_sync_batchnorm()
        ws = torch.zeros(4096, dtype=torch.uint8)
        model._ws = ws
        off = 256
        ws[off:off + 8 * 3 * M].view(torch.float64).copy_(_bn_sums(part, M))
        rc = model._allreduce_cb(ws.data_ptr() + off, 3 * M, None, None)
        sums = ws[off:off + 8 * 3 * M].view(torch.float64).numpy()
        # finalise from the merged sums exactly like tp_fused.h bn_coef, compare with the oracle
        # BatchNorm on the full batch
        n = 40.0
        mu = sums[:M] / n
        var = sums[M:2 * M] / n - mu ** 2
        nv = sums[2 * M:] / (3 * n)
        _, rm, rv = batch_norm(full, Irreps(f"{M}x0e+{M}x1o"), np.ones(2 * M), np.zeros(M), np.zeros(M),
                               np.ones(2 * M), True, momentum=1.0)
        ok = rc == 0 and np.allclose(mu, rm, rtol=1e-12, atol=1e-12) and \
            np.allclose(np.concatenate([var, nv]), rv, rtol=1e-12, atol=1e-12)
        q.put((rank, bool(ok)))
        del ctypes
    finally:
        dist.destroy_process_group()


def test_syncbn_merges_partial_sums_over_gloo():
    """The SEGNN SyncBN hook (segnn.py _allreduce_cb, called by the library between the
    producing and the finalising kernel) turns each rank's partial BatchNorm sums into the
    full-batch sums: the finalised mean / variance / vector norm equal the oracle BatchNorm
    (e3nn semantics) over the whole batch."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_syncbn_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok in res), res


class _RankModel(torch.nn.Module):
    """CPU stand-in with the rollout contract: pos += 0.1 per step, vel = -vel."""

    def rollout(self, loc, vel, mass, T, absolute=False):
        tp, tv = [loc], [vel]
        for _ in range(T - 1):
            tp.append(tp[-1] + 0.1)
            tv.append(-tv[-1])
        return torch.stack(tp, 1), torch.stack(tv, 1)


def _sharded_inference_worker(rank, world, port, out_root, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import numpy as np
    import torch.distributed as dist

    import nbody_amd.dataset as D
    import nbody_amd.inference as I
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def sample(self, batch_size, T=10000, sample_freq=10, seeds=None, shard=False):
            # trajectory i of this rank's shard starts at the GLOBAL system id of that trajectory
            start, _ = shard_range(7, dist.get_rank(), dist.get_world_size())
            Ts = T // sample_freq
            return [(np.full((Ts, 3, 3), float(start + i)), np.zeros((Ts, 3, 3)), np.zeros((Ts, 3, 3)),
                     np.ones((3, 1))) for i in range(batch_size)]
        D.GravitySim.sample_trajectory_batch = sample
        ds = D.GravityDatasetOtf.__new__(D.GravityDatasetOtf)
        ds.batch_size, ds.double_precision, ds.target = 7, True, "pos_dt+vel"
        ds.get_ground_truth_trajectories = lambda batch_size=None, seeds=None, shard=None: (
            sample(None, batch_size, 50, 10), {})
        out_dir, locs, vels = I.run_inference("segnn", None, model=_RankModel(), dataset=ds, device="cpu",
                                              save_dir=os.path.join(out_root, "o"), max_rollout_steps=4,
                                              print_step=False)
        ok = locs.shape == (2, 7, 4, 3, 3)
        ok &= bool(np.array_equal(locs[0][:, 0, 0, 0], np.arange(7.0)))          # ground truth in system order
        ok &= bool(np.allclose(locs[1][:, 3, 0, 0], np.arange(7.0) + 0.3))       # predictions in system order
        files = sorted(os.listdir(out_dir)) if rank == 0 else None
        q.put((rank, ok, files))
    finally:
        dist.destroy_process_group()


def test_sharded_run_inference_reassembles_in_order(tmp_path):
    """run_inference under torch.distributed: each rank generates and rolls out its block of
    systems; one all-gather reassembles [2, B, T, N, 3] in system order on every rank and rank
    0 writes the per-simulation files."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_inference_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res), res
    assert len(res[0][2]) == 4 * 7


# ------------------------------------------------------------------ data-parallel gradients
def _grad_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from nbody_amd import parallel as P
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        lin = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.Tanh(), torch.nn.Linear(7, 3)).double()
        x = torch.randn(8 * world, 5, dtype=torch.float64)
        y = torch.randn(8 * world, 3, dtype=torch.float64)
        sl = slice(8 * rank, 8 * rank + 8)
        torch.nn.functional.mse_loss(lin(x[sl]), y[sl]).backward()
        P.allreduce_gradients(lin.parameters(), bucket_bytes=100)   # several buckets
        q.put((rank, [p.grad.numpy().copy() for p in lin.parameters()]))   # by value: the sender exits
    finally:
        dist.destroy_process_group()


def test_allreduce_gradients_equals_full_batch_mean_over_gloo():
    """Each rank's mean-loss gradient on its shard, averaged over ranks, equals the full-batch
    gradient (equal shards) -- the data-parallel step bench.py --model egnn_mc_train takes."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_grad_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    torch.manual_seed(0)
    lin = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.Tanh(), torch.nn.Linear(7, 3)).double()
    x = torch.randn(8 * world, 5, dtype=torch.float64)
    y = torch.randn(8 * world, 3, dtype=torch.float64)
    torch.nn.functional.mse_loss(lin(x), y).backward()
    for r in range(world):
        for g, p in zip(res[r], lin.parameters()):
            torch.testing.assert_close(torch.from_numpy(g), p.grad, rtol=1e-12, atol=1e-14)
