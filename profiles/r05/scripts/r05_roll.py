"""Diagnosis: the C2 rollout fixture (tests/test_gpu_segnn.py::test_rollout_c2_matches_oracle_fixture)
under several path settings, one spawned child each: per-step MSE against the fp64 oracle and the
systems with the largest error at each step past the predictable horizon."""
import multiprocessing as mp
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def child(env, q):
    os.environ.update(env)
    import torch
    import nbody_amd.segnn as S
    fx = np.load(os.path.join(ROOT, "tests", "golden", "segnn_c2_rollout.npz"))
    torch.manual_seed(0)
    dev = torch.device("cuda:0")
    model = S.SEGNN(hidden_features=192, num_layers=6).to(dev).train()
    t = lambda a: torch.tensor(a, dtype=torch.float32, device=dev)
    T = fx["traj_loc"].shape[1]
    tp, tv = model.rollout(t(fx["loc0"]), t(fx["vel0"]), t(np.ones(fx["loc0"].shape[:2] + (1,))), T)
    q.put((tp.double().cpu().numpy(), tv.double().cpu().numpy()))


if __name__ == "__main__":
    envs = [dict(kv.split("=", 1) for kv in a.split(",")) if a else {} for a in sys.argv[1:]] or [{}]
    fx = np.load(os.path.join(ROOT, "tests", "golden", "segnn_c2_rollout.npz"))
    rl, fl = fx["traj_loc"].astype(np.float64), fx["f32_loc"].astype(np.float64)
    ctx = mp.get_context("spawn")
    res = {}
    for env in envs:
        q = ctx.Queue()
        p = ctx.Process(target=child, args=(env, q))
        p.start()
        tp, tv = q.get(timeout=300)
        p.join(timeout=60)
        tag = ",".join(f"{k}={os.path.basename(v)}" for k, v in env.items()) or "default"
        res[tag] = tp
        line = []
        for k in range(1, tp.shape[1]):
            mse = float(((tp[:, k] - rl[:, k]) ** 2).mean())
            line.append(f"{mse:.1e}")
        pl_ = fx["pert_loc"].astype(np.float64)
        stats = []
        for k in range(6, tp.shape[1]):
            sc = np.abs(rl[:, k]).max()
            per = lambda a: np.abs(a[:, k] - rl[:, k]).reshape(a.shape[0], -1).max(1) / sc
            e_dev, e_f32, e_pert = per(tp), per(fl), per(pl_)
            e_ref = np.maximum(e_f32, e_pert)
            ok = float(np.mean(e_dev <= 10 * e_ref + 1e-6))
            stats.append(f"k{k}: ok {ok:.4f} med {np.median(e_dev):.1e}/{np.median(e_f32):.1e}")
        print(f"{tag}: " + "; ".join(stats), flush=True)
        err = ((tp[:, 6] - rl[:, 6]) ** 2).reshape(tp.shape[0], -1).sum(1)
        worst = np.argsort(err)[::-1][:4]
        print(f"{tag}: MSE per step {' '.join(line)}; step 6 worst systems {worst.tolist()} "
              f"({', '.join(f'{err[w]:.2e}' for w in worst)})", flush=True)
    f32 = [f"{float(((fl[:, k] - rl[:, k]) ** 2).mean()):.1e}" for k in range(1, rl.shape[1])]
    err = ((fl[:, 6] - rl[:, 6]) ** 2).reshape(fl.shape[0], -1).sum(1)
    print(f"fp32 oracle: MSE per step {' '.join(f32)}; step 6 worst systems {np.argsort(err)[::-1][:4].tolist()}")
