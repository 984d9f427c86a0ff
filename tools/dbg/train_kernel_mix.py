"""Kernel mix of one eager training step (forward + MSE + backward) per model: the device kernels
torch.profiler records, split into libnbx kernels and torch kernels (elementwise glue, fills, copies,
reductions), with counts and summed device time.  Usage: python tools/dbg/train_kernel_mix.py [models]"""
import collections
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402

dev = torch.device("cuda:0")


class _G:
    pass


def segnn():
    import nbody_amd.segnn as S
    from nbody_amd.graph import fc_edge_index
    B, N = 64, 5
    torch.manual_seed(0)
    m = S.SEGNN(hidden_features=bench.HIDDEN, num_layers=bench.LAYERS).to(dev).train()
    loc, vel, mass = bench.initial_states(B, N, 0)
    t = lambda x: torch.tensor(x, dtype=torch.float32, device=dev)
    g = _G()
    g.pos, g.vel, g.mass = t(loc.reshape(-1, 3)), t(vel.reshape(-1, 3)), t(mass.reshape(-1, 1))
    g.edge_index = fc_edge_index(B, N, dev)
    g.nbx_system_size = N
    return m, (lambda: m(g)), t(np.random.default_rng(1).standard_normal((B * N, 6)) * 0.1)


def ponita():
    import nbody_amd.ponita as PO
    from nbody_amd.graph import build_graph_with_knn
    B, N = 64, 5
    torch.manual_seed(0)
    m = PO.PONITA_NBODY(**bench.PONITA_TRAIN).to(dev).train()
    m.model.materialize()
    loc, vel, mass = bench.initial_states(B, N, 0)
    t = lambda x: torch.tensor(x, dtype=torch.float32, device=dev)
    g = _G()
    g.pos, g.vec, g.x = t(loc.reshape(-1, 3)), t(vel.reshape(-1, 1, 3)), t(mass.reshape(-1, 1))
    g.edge_index = build_graph_with_knn(g.pos, B, N, dev, N - 1)
    g.nbx_system_size = N
    return m, (lambda: m(g)), t(np.random.default_rng(1).standard_normal((B * N, 6)) * 0.1)


def eqv2():
    from nbody_amd.equiformer_v2 import EquiformerV2_nbody
    import nbody_amd.eqv2_train as ET
    B, N = 64, 5
    torch.manual_seed(0)
    m = EquiformerV2_nbody(**bench.EQV2_C4).to(dev).train()
    loc, vel, mass = bench.initial_states(B, N, 0)
    t = lambda x: torch.tensor(x, dtype=torch.float32, device=dev)
    pos, vv, q = t(loc.reshape(-1, 3)), t(vel.reshape(-1, 3)), t(mass.reshape(-1))
    gauge = t(np.random.default_rng(0).uniform(0, 1, (B * N * (N - 1), 3)))
    return m, (lambda: ET.train_forward(m, pos, vv, q, B, N, gauge, 0)), \
        t(np.random.default_rng(1).standard_normal((B * N, 6)) * 0.1)


for name in (sys.argv[1:] or ["segnn", "ponita", "eqv2"]):
    model, fwd, target = {"segnn": segnn, "ponita": ponita, "eqv2": eqv2}[name]()

    def step():
        model.zero_grad(set_to_none=True)
        torch.nn.functional.mse_loss(fwd(), target).backward()
    step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        step()
        torch.cuda.synchronize()
    by = collections.defaultdict(lambda: [0, 0.0])
    for ev in prof.events():
        if ev.device_type.name != "CUDA":
            continue
        k = ev.name
        key = ("torch " + k.split("<")[0].split("(")[0][-60:]) if "at::native" in k or "at::" in k else ("nbx " + k.split("(")[0][-60:])
        by[key][0] += 1
        by[key][1] += ev.device_time_total if hasattr(ev, "device_time_total") else ev.cuda_time_total
    tot_n = sum(v[0] for v in by.values())
    tot_t = sum(v[1] for v in by.values())
    tn = sum(v[0] for k, v in by.items() if k.startswith("torch"))
    tt = sum(v[1] for k, v in by.items() if k.startswith("torch"))
    print(f"== {name}: {tot_n} kernels, {tot_t / 1e3:.2f} ms device; torch glue {tn} kernels, {tt / 1e3:.2f} ms")
    for k, (n, us) in sorted(by.items(), key=lambda kv: -kv[1][1])[:18]:
        print(f"  {n:5d} {us / 1e3:8.3f} ms  {k}")
