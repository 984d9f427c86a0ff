"""Diagnosis: intermittent corruption of SEGNN C2 forwards.  Each child (one library / path setting)
runs K pairs of forwards, every pair on a new seeded batch, and compares the two results of a pair:
train-mode reruns agree to ~1e-6 relative (fp64 atomic BatchNorm sums), so a system off by more than
1e-3 of the output scale in either call is a corrupted forward.
usage: python scripts/race_pairs.py K "<env>" ["<env>" ...]   (env: A=1,B=2; '' = defaults)
PAIRS_EVAL=1: eval-mode BatchNorm."""
import multiprocessing as mp
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def child(env, K, q):
    os.environ.update(env)
    import torch
    import test_gpu_segnn as T
    dev = torch.device("cuda:0")
    model = T.make_model(192, 6, dev, perturb_bn=False).train(os.environ.get("PAIRS_EVAL") != "1")
    sd0 = {k: v.clone() for k, v in model.state_dict().items()}
    B, N = 1024, 5
    bad = []
    for k in range(K):
        pos, vel, mass = T.states(B, N, seed=1000 + k)
        o = []
        for _ in range(2):
            model.load_state_dict(sd0)
            o.append(T.gpu_forward(model, pos, vel, mass, B, N, dev))
        scale = np.abs(o[0]).max(0)
        rel = (np.abs(o[0] - o[1]) / scale).reshape(B, N, -1).max(axis=(1, 2))
        if rel.max() > 1e-3:
            bad.append((k, float(rel.max()), np.argwhere(rel > 1e-3)[:, 0].tolist()[:6]))
    q.put(bad)


if __name__ == "__main__":
    K = int(sys.argv[1])
    envs = [dict(kv.split("=", 1) for kv in a.split(",")) if a else {} for a in sys.argv[2:]] or [{}]
    ctx = mp.get_context("spawn")
    for env in envs:
        q = ctx.Queue()
        p = ctx.Process(target=child, args=(env, K, q))
        p.start()
        bad = q.get(timeout=1500)
        p.join(timeout=60)
        tag = {k: os.path.basename(v) for k, v in env.items()} or "default"
        print(f"{tag}: {len(bad)} of {K} pairs with a corrupted forward" +
              "".join(f"\n   pair {k}: max rel {m:.3e}, systems {s}" for k, m, s in bad[:8]), flush=True)
