"""Diagnosis: the batch-permutation property of tests/test_gpu_segnn.py under several path switches,
one spawned child per setting (the library reads its switches once per process)."""
import multiprocessing as mp
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def child(env, q):
    os.environ.update(env)
    import numpy as np
    import torch
    import test_gpu_segnn as T
    dev = torch.device("cuda:0")
    res = []
    for mode in ("eval", "train"):
        model = T.make_model(192, 6, dev, perturb_bn=False)
        model.train(mode == "train")
        B, N = 1024, 5
        pos, vel, mass = T.states(B, N, seed=4)
        perm = np.random.default_rng(0).permutation(B)
        idx = (perm[:, None] * N + np.arange(N)).reshape(-1)
        a = T.gpu_forward(model, pos, vel, mass, B, N, dev)
        a2 = T.gpu_forward(model, pos, vel, mass, B, N, dev)
        b = T.gpu_forward(model, pos[idx], vel[idx], mass[idx], B, N, dev)
        d = np.abs(b - a[idx])
        bad = np.argwhere(d > 1e-5 * np.abs(a[idx]) + 1e-6)
        res.append((mode, float(d.max()), len(bad), sorted(set((bad[:, 0] // N).tolist()))[:8],
                    float(np.abs(a2 - a).max())))
    q.put(res)


if __name__ == "__main__":
    envs = [{}, {"NBX_UPD_DV": "0"}, {"NBX_MSG_DV": "0"}, {"NBX_UPD_DV": "0", "NBX_MSG_DV": "0"}]
    if len(sys.argv) > 1:
        envs = [dict(kv.split("=") for kv in a.split(",")) if a else {} for a in sys.argv[1:]]
    ctx = mp.get_context("spawn")
    for env in envs:
        q = ctx.Queue()
        p = ctx.Process(target=child, args=(env, q))
        p.start()
        r = q.get(timeout=300)
        p.join(timeout=60)
        for mode, dmax, nbad, systems, rerun in r:
            print(f"{env or 'default'} {mode}: max |perm diff| {dmax:.3e}, {nbad} bad elements, systems {systems}, "
                  f"rerun diff {rerun:.3e}", flush=True)
