"""Diagnosis: the first SEGNN C2 forward of a fresh process against the second one on the same
input (train-mode BatchNorm: fp64 atomic statistics, so reruns agree to ~1e-6 relative).  One
spawned child per (setting, repeat); reports the systems of a first call that is off by > 1e-3.
usage: python scripts/r05_first.py REPEATS "<env>" ["<env>" ...]   (env: A=1,B=2; '' = defaults)"""
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
    import test_gpu_segnn as T
    dev = torch.device("cuda:0")
    model = T.make_model(192, 6, dev, perturb_bn=False).train(os.environ.get("FIRST_EVAL") != "1")
    B, N = 1024, 5
    pos, vel, mass = T.states(B, N, seed=6)
    sd0 = {k: v.clone() for k, v in model.state_dict().items()}
    outs = []
    for _ in range(3):
        model.load_state_dict(sd0)
        outs.append(T.gpu_forward(model, pos, vel, mass, B, N, dev))
    scale = np.abs(outs[2]).max(0)
    res = []
    for o in outs[:2]:
        rel = (np.abs(o - outs[2]) / scale).reshape(B, N, -1).max(axis=(1, 2))
        res.append((float(rel.max()), np.argwhere(rel > 1e-3)[:, 0].tolist()[:6]))
    q.put(res)


if __name__ == "__main__":
    reps = int(sys.argv[1])
    envs = [dict(kv.split("=", 1) for kv in a.split(",")) if a else {} for a in sys.argv[2:]] or [{}]
    ctx = mp.get_context("spawn")
    for env in envs:
        tag = {k: os.path.basename(v) for k, v in env.items()} or "default"
        nbad = 0
        for r in range(reps):
            q = ctx.Queue()
            p = ctx.Process(target=child, args=(env, q))
            p.start()
            res = q.get(timeout=300)
            p.join(timeout=60)
            (m0, s0), (m1, s1) = res
            if s0 or s1:
                nbad += 1
                print(f"{tag} process {r}: call 0 max rel {m0:.3e} systems {s0}; call 1 max rel {m1:.3e} systems {s1}",
                      flush=True)
        print(f"{tag}: {nbad} of {reps} fresh processes with a corrupted call", flush=True)
