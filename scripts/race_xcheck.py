"""Diagnosis: stale or racing reads across SEGNN C2 forwards.  Each child (one library / path
setting) runs K eval-mode forwards on K different seeded batches in one process; the parent compares
every forward with the fp32-MFMA path (NBX_X3=0: no split precision, no decoupled msg_pre hand-off)
computed the same way in its own child.  Paths differ by float rounding only (<= ~1e-5 relative);
a system off by more than 1e-3 of the output scale is reported.
usage: python scripts/race_xcheck.py K "<env>" ["<env>" ...]   (env: A=1,B=2; '' = defaults)
XCHECK_TRAIN=1: train-mode BatchNorm (batch statistics over the 1024 systems)."""
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
    model = T.make_model(192, 6, dev, perturb_bn=False).train(os.environ.get("XCHECK_TRAIN") == "1")
    B, N = 1024, 5
    outs = []
    for k in range(K):
        pos, vel, mass = T.states(B, N, seed=100 + k)
        outs.append(T.gpu_forward(model, pos, vel, mass, B, N, dev).astype(np.float32))
    q.put(np.stack(outs))


def run(env, K):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=child, args=(env, K, q))
    p.start()
    r = q.get(timeout=900)
    p.join(timeout=60)
    return r


if __name__ == "__main__":
    K = int(sys.argv[1])
    envs = [dict(kv.split("=", 1) for kv in a.split(",")) if a else {} for a in sys.argv[2:]]
    ref = run({"NBX_X3": "0"}, K)
    scale = np.abs(ref).reshape(K, -1, ref.shape[-1]).max(1, keepdims=True)   # per call and column
    for env in envs:
        got = run(env, K)
        rel = (np.abs(got - ref).reshape(K, -1, ref.shape[-1]) / scale).reshape(K, 1024, 5, -1).max(axis=(2, 3))
        bad = np.argwhere(rel > 1e-3)
        tag = {k: os.path.basename(v) for k, v in env.items()} or "default"
        print(f"{tag}: max rel {rel.max():.3e}, median over calls of the worst system {np.median(rel.max(1)):.3e}; "
              f"{len(bad)} (call, system) pairs off by > 1e-3" +
              "".join(f"\n   call {c} system {s}: {rel[c, s]:.3e}" for c, s in bad[:8]), flush=True)
