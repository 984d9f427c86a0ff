"""Tuning aid: eager vs hipGraph-replayed SEGNN C2 forwards (per-launch overhead check)."""
import sys
import time

import torch

sys.path.insert(0, ".")
import tests.test_gpu_segnn as T  # noqa: E402
import nbody_amd.graph as G  # noqa: E402

dev = torch.device("cuda:0")
model = T.make_model(192, 6, dev, perturb_bn=False).eval()
B, N = 1024, 5
pos, vel, mass = T.states(B, N, seed=3)
g = T.Graph()
g.pos = torch.tensor(pos, dtype=torch.float32, device=dev)
g.vel = torch.tensor(vel, dtype=torch.float32, device=dev)
g.mass = torch.tensor(mass, dtype=torch.float32, device=dev)
g.edge_index = G.fc_edge_index(B, N, dev)
s = torch.cuda.Stream()
with torch.no_grad(), torch.cuda.stream(s):
    for _ in range(5):
        out = model(g)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        out = model(g)
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / 200
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        out2 = model(g)
    graph.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        graph.replay()
    torch.cuda.synchronize()
    gr = (time.perf_counter() - t0) / 200
print(f"eager {eager*1e6:.1f} us/forward, graph {gr*1e6:.1f} us/forward, max|diff| {(out - out2).abs().max().item():.2e}")
