#!/usr/bin/env python
"""Headline benchmark: SEGNN self-feed rollout steps/sec (BASELINE.json, config C2).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)

Workload (per rank): SEGNN lmax_h=1, hidden_features=192, 6 layers, N=5 bodies,
batch B=1024 systems, fp32, train-mode BatchNorm (the reference rollout never
calls model.eval()).  A "step" = one self-feed model step for the whole batch:
featurise -> SEGNN forward -> state update -> trajectory frame write, all
device-resident (infer_self_feed.py:99-194).  Initial states = frame 0 of
GravitySim(N=5) trajectories with seeds rank*B .. rank*B+B-1; weights from
torch.manual_seed(0).  Multi-GPU: every rank runs its own B=1024 batch (the
reference configuration, BatchNorm statistics per rank), "weak" scaling; the
final states are all-gathered over RCCL inside the timed region.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HIDDEN, LAYERS, NBODY, BATCH = 192, 6, 5, 1024
HBM_PEAK_GBS = 8000.0
FP32_MFMA_PEAK_TFLOPS = 157.3          # MI355X_MICROARCH.md: FP32 matrix (= vector) peak
SURVEY_GFLOP_PER_STEP = 67.73          # algorithmic work of the reference formulation


def useful_gemm_flops(V, E, M, layers):
    """Useful (non-zero-block) MACs x2 of the dominant GEMM kernel per forward, i.e.
    the O(3) tensor-product contractions of the factorised formulation
    (DESIGN.md §Measurement)."""
    per_layer = (
        2 * V * M * 6 * M + 2 * 3 * V * M * 6 * M                    # node_pre (message_layer_1 halves)
        + 2 * E * (2 * M * 2 * M + M * M) + 2 * 3 * E * M * M       # message_layer_2
        + 2 * V * (4 * M * 2 * M + 2 * M * M) + 2 * 3 * V * 2 * M * M  # update_layer_1
        + 2 * V * (2 * M * M + M * M) + 2 * 3 * V * M * M           # update_layer_2
    )
    pre_pool1 = 2 * V * (2 * M * 2 * M + M * M) + 2 * 3 * V * M * M
    return layers * per_layer + pre_pool1


def initial_states(B, N, seed0):
    from nbody_amd.gravity import GravitySim
    sim = GravitySim(n_balls=N, interaction_strength=2, dt=0.01, softening=0.2, device="cpu")
    loc = np.empty((B, N, 3))
    vel = np.empty((B, N, 3))
    for b in range(B):
        p, v, _ = sim.initial_conditions(seed0 + b)
        loc[b], vel[b] = p, v
    return loc, vel, np.ones((B, N, 1))


def cpu_baseline(loc, vel, mass, steps=1):
    """The CPU oracle (numpy fp64 restatement of the reference SEGNN path) timed on
    the host cores on a bounded sample: `steps` self-feed steps of the full B=1024
    batch."""
    from oracle.rollout import rollout, segnn_step
    from oracle.segnn import SEGNNOracle, init_params
    om = SEGNNOracle(hidden_features=HIDDEN, num_layers=LAYERS)
    params = init_params(om, seed=0)
    t0 = time.perf_counter()
    rollout(segnn_step(om, params), loc, vel, np.zeros_like(loc), mass, steps + 1)
    dt = time.perf_counter() - t0
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return {"value": steps / dt, "unit": "steps/s", "cores": threads, "kind": "port",
            "sample": f"{steps} self-feed step(s) of the B={loc.shape[0]} N={loc.shape[1]} batch, numpy fp64 oracle "
                      f"(oracle/segnn.py), BLAS threads={threads}, {dt:.2f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=BATCH)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=1)
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    device = torch.device("cuda", local)

    import nbody_amd.segnn as S
    from nbody_amd import _lib

    B, N = a.batch, NBODY
    torch.manual_seed(0)
    model = S.SEGNN(hidden_features=HIDDEN, num_layers=LAYERS, lmax_h=1).to(device).float().train()
    loc, vel, mass = initial_states(B, N, rank * B)
    loc_d = torch.tensor(loc, dtype=torch.float32, device=device)
    vel_d = torch.tensor(vel, dtype=torch.float32, device=device)
    mass_d = torch.tensor(mass, dtype=torch.float32, device=device)

    # warmup (also packs weights / allocates the workspace)
    if a.warmup > 0:
        model.rollout(loc_d, vel_d, mass_d, a.warmup + 1)
    torch.cuda.synchronize(device)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    tp, tv = model.rollout(loc_d, vel_d, mass_d, a.steps + 1)
    final = torch.cat([tp[:, -1], tv[:, -1]], -1).contiguous()
    if dist:
        gathered = [torch.empty_like(final) for _ in range(world)]
        dist.all_gather(gathered, final)
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    finite = bool(torch.isfinite(tp).all().item())

    # live roofline of the dominant kernel (tp_fused_kernel): HIP events around
    # every GEMM launch of a few forwards on the launch stream
    V, E, M = B * N, B * N * (N - 1), model.mul
    p32 = loc_d.reshape(-1, 3).contiguous()
    v32 = vel_d.reshape(-1, 3).contiguous()
    m32 = mass_d.reshape(-1).contiguous()
    out = torch.empty(V, 6, device=device)
    W = model._weights(device)
    ws = model._workspace(B, N, device)
    g_ms, g_n, g_fl, tot = _lib.c_f(), _lib.c_i32(), _lib.c_d(), _lib.c_f()
    reps, gemm_ms, gemm_launches, fwd_ms = 5, 0.0, 0, 0.0
    for _ in range(reps):
        _lib.check(_lib.lib().nbx_segnn_forward_timed(
            W, _lib.dev_ptr(p32), _lib.dev_ptr(v32), _lib.dev_ptr(m32), B, N, _lib.dev_ptr(out), _lib.dev_ptr(ws),
            ws.numel(), _lib.stream_ptr(device), g_ms, g_n, g_fl, tot), "forward_timed")
        gemm_ms += g_ms.value
        gemm_launches += g_n.value
        fwd_ms += tot.value
    useful = useful_gemm_flops(V, E, M, LAYERS)
    avg_launch_s = gemm_ms / gemm_launches / 1e3
    useful_per_launch = useful / (gemm_launches / reps)
    achieved_tflops = useful_per_launch / avg_launch_s / 1e12

    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_gemm_f32.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            traffic = json.load(f).get("hbm_bytes_per_launch")

    steps_per_s_rank = a.steps / elapsed
    value = steps_per_s_rank * world
    result = {
        "metric": "self-feed rollout steps/sec, SEGNN N=5 batch=1024",
        "value": round(value, 3),
        "unit": "steps/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(1e3 * elapsed / a.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (GravitySim frame-0 initial states, seeded random-init weights)",
        "config": {"workload": "C2: SEGNN lmax_h=1 hidden=192 layers=6, N=5, batch=1024 per GPU, self-feed rollout",
                   "model": "SEGNN", "global_batch": B * world, "seq_len": a.steps, "parallelism": f"dp{world}",
                   "bn_mode": "batch statistics per rank (reference train-mode rollout)"},
        "trajectory_steps_per_s": round(value * B, 1),
        "survey_formulation_tflops": round(value * SURVEY_GFLOP_PER_STEP / 1e3, 3),
        "roofline": {"bound": "mfma", "kernel": "tp_fused_kernel (v_mfma_f32_32x32x2_f32, weight-stationary)",
                     "achieved": round(achieved_tflops, 3), "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved_tflops / FP32_MFMA_PEAK_TFLOPS, 4), "traffic": traffic,
                     "avg_launch_us": round(avg_launch_s * 1e6, 3),
                     "useful_gflop_per_launch": round(useful_per_launch / 1e9, 4),
                     "executed_gflop_per_launch": round(g_fl.value / g_n.value / 1e9, 4),
                     "gemm_share_of_forward": round(gemm_ms / fwd_ms, 3)},
        "finite": finite,
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(loc, vel, mass, a.cpu_steps)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
