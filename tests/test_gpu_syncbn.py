"""SyncBN on the device: two ranks (gloo process group, both on the box's one GPU) each run
the C2-shaped SEGNN (hidden 192, 6 layers) on half of a batch with the BatchNorm sums
all-reduced between the producing and finalising kernels (segnn.py enable_sync_batchnorm,
include/nbx.h bn_allreduce); the halves must reproduce the single-process full-batch
train-mode forward and 3-frame rollout (the reference's statistics over all E edges / V
nodes, models/segnn/segnn.py:233-235,257-261,282-283)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B, N, T = 64, 5, 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs():
    rng = np.random.default_rng(11)
    return rng.standard_normal((B, N, 3)), rng.standard_normal((B, N, 3))


def _model(device, deterministic=False):
    from nbody_amd.segnn import SEGNN
    torch.manual_seed(0)
    return SEGNN(hidden_features=192, num_layers=6, deterministic=deterministic).to(device).train()


def _run(model, loc, vel, device, knn=None):
    import nbody_amd.graph as G

    class Graph:
        pass
    b = loc.shape[0]
    g = Graph()
    g.pos = torch.tensor(loc.reshape(-1, 3), dtype=torch.float32, device=device)
    g.vel = torch.tensor(vel.reshape(-1, 3), dtype=torch.float32, device=device)
    g.mass = torch.ones(b * N, 1, device=device)
    g.edge_index = G.fc_edge_index(b, N, device)
    sd0 = {k: v.clone() for k, v in model.state_dict().items()}
    with torch.no_grad():
        out = model(g).cpu().numpy()
    stats = {k: v.cpu().numpy() for k, v in model.state_dict().items() if "running" in k}
    model.load_state_dict(sd0)
    t = lambda a: torch.tensor(a, dtype=torch.float32, device=device)
    tp, tv = model.rollout(t(loc), t(vel), torch.ones(b, N, 1, device=device), T,
                           **({"num_neighbors": knn} if knn else {}))
    return out, stats, tp.cpu().numpy(), tv.cpu().numpy()


def _worker(rank, world, port, q, backend="gloo", deterministic=False, knn=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist
    dev = torch.device("cuda:0")
    if backend == "nccl":
        torch.cuda.set_device(dev)
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        loc, vel = _inputs()
        sl = slice(rank * B // world, (rank + 1) * B // world)
        model = _model(dev, deterministic).enable_sync_batchnorm()
        assert (model._bn_comm is not None) == (backend == "nccl")
        q.put((rank, _run(model, loc[sl], vel[sl], dev, knn)))
        model.disable_sync_batchnorm()
    except Exception as e:  # surfaced by the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_syncbn_two_ranks_reproduce_full_batch(hip_device):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        assert not isinstance(res[r], str), res[r]
    loc, vel = _inputs()
    out, stats, tp, tv = _run(_model(hip_device), loc, vel, hip_device)
    got_out = np.concatenate([res[0][0], res[1][0]])
    scale = np.abs(out).max(0)
    assert (np.abs(got_out - out).max(0) <= 1e-5 * scale).all()
    for k, v in stats.items():       # every rank updated the running stats with the GLOBAL statistics
        for r in (0, 1):
            np.testing.assert_allclose(res[r][1][k], v, rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(np.concatenate([res[0][2], res[1][2]]), tp, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(np.concatenate([res[0][3], res[1][3]]), tv, rtol=1e-4, atol=1e-5)
    # and without SyncBN the halves differ (per-rank statistics): the test is sensitive
    half = _run(_model(hip_device), loc[:B // 2], vel[:B // 2], hip_device)[0]
    assert np.abs(half - out[:B // 2 * N]).max() > 1e-3 * np.abs(out).max()


def _spawn(world, **kw):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q), kwargs=kw) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert not isinstance(res[r], str), res[r]
    return res


def test_syncbn_knn_rollout_two_ranks_reproduce_full_batch(hip_device):
    """kNN graphs (num_neighbors=2 < N-1, infer_self_feed.py:121-123) under SyncBN: the general-graph
    path reduces each BatchNorm's partial rows in a fixed order, all-reduces the sums and finalises
    them (bn_reduce_kernel / bn_coef_kernel); two half-batch ranks reproduce the single-process
    kNN rollout, whose message-BN count is the global V k."""
    res = _spawn(2, knn=2)
    loc, vel = _inputs()
    _, _, tp, tv = _run(_model(hip_device), loc, vel, hip_device, knn=2)
    np.testing.assert_allclose(np.concatenate([res[0][2], res[1][2]]), tp, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(np.concatenate([res[0][3], res[1][3]]), tv, rtol=1e-4, atol=1e-5)


def test_syncbn_deterministic_two_ranks_bit_reproducible(hip_device):
    """deterministic=True under SyncBN: fixed-order partial-row reductions, then the all-reduce; two
    runs of the sharded forward + rollout are bit-identical and reproduce the full batch."""
    a, b = _spawn(2, deterministic=True), _spawn(2, deterministic=True)
    for r in (0, 1):
        for i in (0, 2, 3):
            np.testing.assert_array_equal(a[r][i], b[r][i])
    loc, vel = _inputs()
    out, _, tp, tv = _run(_model(hip_device, True), loc, vel, hip_device)
    scale = np.abs(out).max(0)
    assert (np.abs(np.concatenate([a[0][0], a[1][0]]) - out).max(0) <= 1e-5 * scale).all()
    np.testing.assert_allclose(np.concatenate([a[0][2], a[1][2]]), tp, rtol=1e-4, atol=1e-5)


def test_syncbn_rccl_communicator_single_rank(hip_device):
    """The library-owned RCCL communicator (nbx_comm_init; enable_sync_batchnorm under the nccl
    backend): the all-reduces are enqueued by libnbx on the launch stream.  One rank (the box has one
    GPU; RCCL refuses two ranks on one device): the sum over one rank is the identity, so the
    deterministic SyncBN forward and rollout equal the plain deterministic ones bit for bit."""
    res = _spawn(1, backend="nccl", deterministic=True)
    loc, vel = _inputs()
    out, stats, tp, tv = _run(_model(hip_device, True), loc, vel, hip_device)
    np.testing.assert_array_equal(res[0][0], out)
    np.testing.assert_array_equal(res[0][2], tp)
    np.testing.assert_array_equal(res[0][3], tv)


class _GtDataset:
    """run_inference's dataset contract (batch_size, double_precision, target,
    get_ground_truth_trajectories): system i of the global batch starts at GravitySim frame 0 of seed i,
    whichever rank holds it (the reference draws unseeded trajectories; fixed seeds make the sharded and
    the single-process rollouts comparable)."""

    def __init__(self, B, T, N=5):
        self.batch_size, self.double_precision, self.target = B, False, "pos_dt+vel"
        self.T, self.N = T, N

    def get_ground_truth_trajectories(self, batch_size=None, seeds=None, shard=None):
        import torch.distributed as dist
        from nbody_amd.parallel import shard_range
        from oracle.gravity import initial_conditions
        world = dist.get_world_size() if dist.is_initialized() else 1
        rank = dist.get_rank() if dist.is_initialized() else 0
        start, _ = shard_range(self.batch_size, rank, world) if batch_size != self.batch_size else (0, 0)
        out = []
        for i in range(batch_size):
            p, v, _ = initial_conditions(self.N, start + i)
            out.append((np.repeat(p[None], self.T, 0), np.repeat(v[None], self.T, 0), np.zeros((self.T, self.N, 3)),
                        np.ones((self.N, 1))))
        return out, {}


def _inference_worker(rank, world, port, q, B, T, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import nbody_amd.inference as I
        model = _model(torch.device("cuda:0"))
        _, locs, vels = I.run_inference("segnn", None, model=model, dataset=_GtDataset(B, T), device="cuda:0",
                                        save_dir=os.path.join(out_dir, f"r{rank}"), max_rollout_steps=T,
                                        print_step=False)
        q.put((rank, (locs[1], vels[1])))
    except Exception as e:  # surfaced by the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_sharded_run_inference_native_segnn_matches_single_process(hip_device, tmp_path):
    """run_inference sharded over two ranks (gloo, both on the box's GPU) with the native SEGNN rollout in
    train mode: each rank rolls out its half of the batch with SyncBN (the reference's full-batch
    BatchNorm statistics), one all-gather reassembles [2, B, T, N, 3]; the predictions equal the
    single-process run_inference of the whole batch."""
    import nbody_amd.inference as I
    B, T = 48, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_inference_worker, args=(r, 2, port, q, B, T, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        assert not isinstance(res[r], str), res[r]
    _, locs, vels = I.run_inference("segnn", None, model=_model(hip_device), dataset=_GtDataset(B, T),
                                    device=hip_device, save_dir=str(tmp_path / "single"), max_rollout_steps=T,
                                    print_step=False)
    for r in (0, 1):
        np.testing.assert_allclose(res[r][0], locs[1], rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(res[r][1], vels[1], rtol=1e-4, atol=1e-5)
    assert np.abs(locs[1][:, 1:] - locs[1][:, :1]).max() > 1e-3    # the rollout moved the bodies


def _train_inputs(b, seed=5):
    rng = np.random.default_rng(seed)
    return (rng.standard_normal((b, N, 3)), rng.standard_normal((b, N, 3)) * 0.3,
            rng.integers(1, 4, (b, N, 1)).astype(np.float64), rng.standard_normal((b * N, 6)) * 0.1)


def _train_step(model, loc, vel, mass, tgt, device):
    """One grad-mode forward (the native training operators) + MSE loss + backward -> (pred, loss,
    grads, running stats)."""
    import nbody_amd.graph as G

    class Graph:
        pass
    b = loc.shape[0]
    g = Graph()
    g.pos = torch.tensor(loc.reshape(-1, 3), dtype=torch.float32, device=device)
    g.vel = torch.tensor(vel.reshape(-1, 3), dtype=torch.float32, device=device)
    g.mass = torch.tensor(mass.reshape(-1, 1), dtype=torch.float32, device=device)
    g.edge_index = G.fc_edge_index(b, N, device)
    model.zero_grad(set_to_none=True)
    pred = model(g)
    loss = torch.nn.functional.mse_loss(pred, torch.tensor(tgt, dtype=torch.float32, device=device))
    loss.backward()
    grads = {k: p.grad.double().cpu().numpy() for k, p in model.named_parameters() if p.grad is not None}
    stats = {k: v.double().cpu().numpy() for k, v in model.state_dict().items() if "running" in k}
    return pred.detach().double().cpu().numpy(), float(loss.detach()), grads, stats


def _train_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist
    from nbody_amd.segnn import SEGNN
    dev = torch.device("cuda:0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        loc, vel, mass, tgt = _train_inputs(B)
        sl = slice(rank * B // world, (rank + 1) * B // world)
        torch.manual_seed(0)
        model = SEGNN(hidden_features=64, num_layers=3).to(dev).train().enable_sync_batchnorm()
        pred, loss, grads, stats = _train_step(model, loc[sl], vel[sl], mass[sl], tgt[sl.start * N:sl.stop * N], dev)
        from nbody_amd.parallel import allreduce_gradients
        allreduce_gradients(list(model.parameters()))             # data-parallel average
        avg = {k: p.grad.double().cpu().numpy() for k, p in model.named_parameters() if p.grad is not None}
        q.put((rank, (pred, loss, avg, stats)))
        model.disable_sync_batchnorm()
    except Exception as e:  # surfaced by the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_syncbn_training_step_two_ranks_reproduce_full_batch(hip_device):
    """Sharded SEGNN training step with SyncBN (segnn_train._SyncBNFn: nbx_bn_train_sums -> all-reduce of
    the fp64 sums and row count -> nbx_bn_train_apply, and the same for the backward sums): two gloo
    ranks on half batches each, gradients averaged over the ranks, reproduce the single-process
    full-batch step -- predictions, the (equal-halves) mean loss, every parameter gradient and the
    running statistics (the reference trains on one device with the statistics of the whole batch,
    trainer.py:233-358)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_train_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        assert not isinstance(res[r], str), res[r]
    from nbody_amd.segnn import SEGNN
    loc, vel, mass, tgt = _train_inputs(B)
    torch.manual_seed(0)
    model = SEGNN(hidden_features=64, num_layers=3).to(hip_device).train()
    pred, loss, grads, stats = _train_step(model, loc, vel, mass, tgt, hip_device)
    got = np.concatenate([res[0][0], res[1][0]])
    scale = np.abs(pred).max(0)
    assert (np.abs(got - pred).max(0) <= 1e-5 * scale + 1e-7).all(), np.abs(got - pred).max(0) / scale
    assert abs(0.5 * (res[0][1] + res[1][1]) - loss) <= 1e-5 * abs(loss)
    for k, g in grads.items():
        for r in (0, 1):   # both ranks hold the averaged gradient
            e = np.abs(res[r][2][k] - g).max()
            assert e <= 2e-4 * np.abs(g).max() + 1e-7, (k, e, np.abs(g).max())
    for k, v in stats.items():
        for r in (0, 1):
            np.testing.assert_allclose(res[r][3][k], v, rtol=1e-5, atol=1e-7)


def _bn_empty_worker(rank, world, port, q):
    """Rank 0 holds every row, rank 1 none: both must reach each all-reduce of _SyncBNFn."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist
    from nbody_amd.segnn_train import _SyncBNFn
    dev = torch.device("cuda:0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        S, V, w, b, dOS, dOV = _bn_inputs(dev)
        if rank == 1:
            S, V, dOS, dOV = S[:0], V[:, :0], dOS[:0], dOV[:, :0]
        S.requires_grad_(True); V.requires_grad_(True); w.requires_grad_(True); b.requires_grad_(True)
        rm, rv = torch.zeros(S.shape[1], device=dev), torch.ones(2 * S.shape[1], device=dev)
        OS, OV = _SyncBNFn.apply(S, V, w, b, rm, rv, 1e-5, 0.1, dist.group.WORLD)
        torch.autograd.backward([OS, OV], [dOS, dOV])
        q.put((rank, [t.detach().cpu().numpy() for t in (OS, OV, S.grad, V.grad, w.grad, b.grad, rm, rv)]))
    except Exception as e:
        import traceback
        q.put((rank, repr(e) + traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def _bn_inputs(dev, rows=200, M=32):
    g = torch.Generator().manual_seed(5)
    mk = lambda *s: torch.randn(*s, generator=g).to(dev)
    return mk(rows, M), mk(3, rows, M), mk(2 * M) + 1.0, mk(M), mk(rows, M), mk(3, rows, M)


def test_syncbn_training_bn_with_an_empty_shard(hip_device):
    """A rank whose shard has no rows (uneven last batch, batch smaller than the world) still takes
    part in _SyncBNFn's forward and backward all-reduces (nbx_bn_train_sums / _apply / _backward_apply
    accept rows == 0); the rank with all rows reproduces the single-process batch-statistics
    BatchNorm (_BNFn): outputs, input and parameter gradients, running statistics."""
    from nbody_amd.segnn_train import _BNFn
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bn_empty_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        assert not isinstance(res[r], str), res[r]
    S, V, w, b, dOS, dOV = _bn_inputs(hip_device)
    for t in (S, V, w, b):
        t.requires_grad_(True)
    rm, rv = torch.zeros(S.shape[1], device=hip_device), torch.ones(2 * S.shape[1], device=hip_device)
    OS, OV = _BNFn.apply(S, V, w, b, rm, rv, 1e-5, 0.1)
    torch.autograd.backward([OS, OV], [dOS, dOV])
    ref = [t.detach().cpu().numpy() for t in (OS, OV, S.grad, V.grad, w.grad, b.grad, rm, rv)]
    for got, want in zip(res[0], ref):
        np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-5)
    assert res[1][0].shape == (0, S.shape[1]) and res[1][2].shape == (0, S.shape[1])
    # the empty rank still updates its running statistics with the global batch statistics
    np.testing.assert_allclose(res[1][6], ref[6], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(res[1][7], ref[7], rtol=1e-5, atol=1e-6)
    # its parameter gradients are zero (no local rows); the data-parallel all-reduce sums them
    np.testing.assert_array_equal(res[1][4], 0.0)
    np.testing.assert_array_equal(res[1][5], 0.0)
