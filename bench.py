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

    # live roofline of the dominant kernel: HIP events around every launch of the
    # fused tensor-product kernels of a few forwards, on the launch stream, split by kind
    V, M = B * N, model.mul
    p32 = loc_d.reshape(-1, 3).contiguous()
    v32 = vel_d.reshape(-1, 3).contiguous()
    m32 = mass_d.reshape(-1).contiguous()
    out = torch.empty(V, 6, device=device)
    W = model._weights(device)
    ws = model._workspace(B, N, device)
    kms, kn, kfl, tot = (_lib.c_f * 4)(), (_lib.c_i32 * 4)(), (_lib.c_d * 4)(), _lib.c_f()
    reps = 5
    ms_k, n_k, fl_k, fwd_ms = [0.0] * 4, [0] * 4, [0.0] * 4, 0.0
    for _ in range(reps):
        _lib.check(_lib.lib().nbx_segnn_forward_timed(
            W, _lib.dev_ptr(p32), _lib.dev_ptr(v32), _lib.dev_ptr(m32), B, N, _lib.dev_ptr(out), _lib.dev_ptr(ws),
            ws.numel(), _lib.stream_ptr(device), kms, kn, kfl, tot), "forward_timed")
        for k in range(4):
            ms_k[k] += kms[k]
            n_k[k] += kn[k]
            fl_k[k] += kfl[k]
        fwd_ms += tot.value
    # rocprofv3 names of the four fused TP launch kinds (csrc/segnn.hip::forward_impl)
    names = ["void nbx::tp16_kernel<3, 0, 0, 2>(nbx::TpProb)", "void nbx::tp_fused_kernel<3, 1, 1>(nbx::TpProb)",
             "void nbx::tp16_kernel<3, 1, 2, 1>(nbx::TpProb)", "void nbx::tp16_kernel<2, 1, 3, 2>(nbx::TpProb)"]
    roles = ["message_layer_1 node halves", "message_layer_2 + gate + aggregation + BN sums",
             "update_layer_1 + gate (pre_pool1 uses CG=2)", "update_layer_2 + residual + BN sums"]
    per_kind = {}
    for k in range(4):
        if n_k[k]:
            avg_s = ms_k[k] / n_k[k] / 1e3
            fl = fl_k[k] / n_k[k]
            per_kind[names[k]] = {"role": roles[k], "avg_launch_us": round(avg_s * 1e6, 3), "gflop_per_launch": round(fl / 1e9, 4),
                                  "tflops": round(fl / avg_s / 1e12, 3), "share_of_forward": round(ms_k[k] / fwd_ms, 3)}
    dom = max(range(4), key=lambda k: ms_k[k])
    dom_avg_s = ms_k[dom] / n_k[dom] / 1e3
    dom_flops = fl_k[dom] / n_k[dom]
    achieved_tflops = dom_flops / dom_avg_s / 1e12
    fused_share = sum(ms_k) / fwd_ms

    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_tp_kernels.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            traffic = json.load(f)["kernels"].get(names[dom], {}).get("hbm_bytes_per_launch")

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
        "roofline": {"bound": "mfma", "kernel": names[dom], "achieved": round(achieved_tflops, 3),
                     "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved_tflops / FP32_MFMA_PEAK_TFLOPS, 4), "traffic": traffic,
                     "avg_launch_us": round(dom_avg_s * 1e6, 3), "gflop_per_launch": round(dom_flops / 1e9, 4),
                     "fused_tp_share_of_forward": round(fused_share, 3), "per_kind": per_kind},
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
