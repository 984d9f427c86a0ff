"""Time the native EquiformerV2 forward / rollout step at the C4 size (B = 256, N = 20)."""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from nbody_amd.equiformer_v2 import EquiformerV2_nbody  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--nodes", type=int, default=20)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--frames", type=int, default=11)
a = ap.parse_args()
cfg = json.load(open(os.path.join(ROOT, "tests", "golden", "eqv2_state.json")))["c4"]["config"]
dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = EquiformerV2_nbody(**cfg).to(dev).eval()
B, N = a.batch, a.nodes
loc = torch.randn(B, N, 3, device=dev)
vel = torch.randn(B, N, 3, device=dev) * 0.3
mass = torch.ones(B, N, 1, device=dev)
batch = torch.arange(B, device=dev).repeat_interleave(N)
x = (loc.reshape(-1, 3), vel.reshape(-1, 3), torch.zeros(B * N, 3, device=dev), mass.reshape(-1, 1), loc.reshape(-1, 3))
for _ in range(3):
    m(x, batch)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(a.iters):
    m(x, batch)
torch.cuda.synchronize()
ms = (time.perf_counter() - t) / a.iters * 1e3
print(f"forward B={B} N={N}: {ms:.3f} ms  ({1e3 / ms:.1f} steps/s)", flush=True)
m.rollout(loc, vel, mass, 3)
torch.cuda.synchronize()
t = time.perf_counter()
m.rollout(loc, vel, mass, a.frames)
torch.cuda.synchronize()
ms = (time.perf_counter() - t) / (a.frames - 1) * 1e3
print(f"rollout step B={B} N={N}: {ms:.3f} ms  ({1e3 / ms:.1f} steps/s)", flush=True)
