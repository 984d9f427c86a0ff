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


def _model(device):
    from nbody_amd.segnn import SEGNN
    torch.manual_seed(0)
    return SEGNN(hidden_features=192, num_layers=6).to(device).train()


def _run(model, loc, vel, device):
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
    tp, tv = model.rollout(t(loc), t(vel), torch.ones(b, N, 1, device=device), T)
    return out, stats, tp.cpu().numpy(), tv.cpu().numpy()


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        loc, vel = _inputs()
        sl = slice(rank * B // world, (rank + 1) * B // world)
        model = _model(dev).enable_sync_batchnorm()
        q.put((rank, _run(model, loc[sl], vel[sl], dev)))
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
