"""Multi-rank rehearsal of bench.py's sharded lines (the driver's N = 2..8 scaling runs): two ranks
of a gloo process group, both on the box's one GPU (parallel.init_from_env with NBX_LOCAL_DEVICE /
NBX_DIST_BACKEND), run the strong-scaling bench functions on halves of one global batch.  The
all-gathered final states must equal a one-rank run of the same global batch, so the per-rank
seeds, the shard ranges, the padding of uneven shards and PONITA's one-time calibration over the
global batch are right before SCALE runs them on eight GPUs (the reference integrates and rolls
out every system independently: helper_scripts/infer_self_feed.py:99-194,
datasets/nbody/dataset/synthetic_sim.py:357-420)."""
import argparse
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _args(model, batch, steps, warmup):
    return argparse.Namespace(model=model, batch=batch, steps=steps, warmup=warmup, no_cpu_baseline=True,
                              cpu_steps=1, cpu_torch_steps=1, eager=False, deterministic_bn=False, bn_mode="batch",
                              gpus=1)


def _bench(model, a, rank, world):
    sys.path.insert(0, ROOT)
    import bench
    from nbody_amd import parallel as P
    rk, ws, dev = P.init_from_env()
    assert (rk, ws) == (rank, world)
    fn = {"ponita": bench.bench_ponita, "gravity": bench.bench_gravity}[model]
    res = fn(a, rk, ws, dev, P)
    return res, a.final_states.double().cpu().numpy()


def _worker(rank, world, port, q, model, a):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), NBX_LOCAL_DEVICE="0", NBX_DIST_BACKEND="gloo",
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist
    try:
        res, final = _bench(model, a, rank, world)
        q.put((rank, (res["value"], res["n_gpus"], final)))
    except Exception as e:  # surfaced by the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _sharded(model, a, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, model, a)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert not isinstance(res[r], str), res[r]
    return res


def _single(model, a):
    """The same bench function as one rank (its own process: the bench's module state stays apart)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(0, 1, _free_port(), q, model, a))
    p.start()
    r = q.get(timeout=300)
    p.join(timeout=60)
    assert not isinstance(r[1], str), r[1]
    return r[1]


def test_gravity_bench_two_ranks_equal_one_rank(hip_device):
    """C5 strong scaling: 25 systems (N = 100) over two ranks (13 + 12: an uneven, padded gather);
    the gathered final positions / velocities equal the one-rank run bit for bit."""
    a = _args("gravity", batch=25, steps=20, warmup=10)
    res = _sharded("gravity", a)
    one = _single("gravity", a)
    assert res[0][1] == 2 and one[1] == 1
    for r in (0, 1):       # every rank holds the whole gathered batch
        assert res[r][2].shape == (25, 100, 6)
        np.testing.assert_array_equal(res[r][2], one[2])


def test_ponita_bench_two_ranks_equal_one_rank(hip_device):
    """C3 strong scaling (PONITA hidden 128, 6 layers, 20 orientations): 66 systems over two ranks;
    the calibration runs on the moments of the whole global batch, so the gathered final states
    equal the one-rank run (up to the fp64 order of the calibration moments, rtol 1e-6)."""
    a = _args("ponita", batch=66, steps=2, warmup=1)
    res = _sharded("ponita", a)
    one = _single("ponita", a)
    for r in (0, 1):
        assert res[r][2].shape == (66, 5, 6)
        np.testing.assert_allclose(res[r][2], one[2], rtol=1e-6, atol=1e-6)
    assert np.isfinite(one[2]).all()
