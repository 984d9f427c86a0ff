#!/usr/bin/env python
"""Headline benchmark: SEGNN self-feed rollout steps/sec (BASELINE.json, config C2).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model segnn|ponita|egnn_mc|gravity]
    (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)

Default (the driver's line) — C2: SEGNN lmax_h=1, hidden_features=192, 6 layers,
N=5 bodies, batch B=1024 systems per rank, fp32, train-mode BatchNorm (the
reference rollout never calls model.eval()).  A "step" = one self-feed model step
for the whole batch: featurise -> SEGNN forward -> state update -> trajectory
frame write, all device-resident (infer_self_feed.py:99-194).  Initial states =
frame 0 of GravitySim(N=5) trajectories with seeds rank*B .. rank*B+B-1; weights
from torch.manual_seed(0).  Multi-GPU: every rank runs its own B=1024 batch (the
reference configuration; BatchNorm statistics per rank), "weak" scaling; the
final states are all-gathered over RCCL inside the timed region.

Secondary configurations (not the headline; same JSON shape):
  --model ponita   C3: PONITA hidden 128, 6 layers, 20 orientations, basis 128, N=5,
                   global batch 4096 sharded over the ranks ("strong" scaling).
  --model egnn_mc  C1: EGNN-MC 6 x 128, N=5, batch 64 per rank ("weak").
  --model eqv2     C4: EquiformerV2 (config.yaml widths), N=20, batch 256 per rank ("weak").
  --model egnn_mc_train  SURVEY 8(f)4: EGNN-MC training step (C1 widths, forward + backward + Adam,
                   gradients all-reduced over ranks), batch 64 per rank ("weak").
  --model segnn_train / ponita_train / eqv2_train  SURVEY 8(f)4: SEGNN (C2 widths) / PONITA
                   (config.yaml: 128 x 8) / EquiformerV2 (C4 widths, N=5) training step, batch 64 per rank.
  --model gravity  C5: ground-truth integrator, 10 000 systems x N=100, --steps
                   KDK steps (sample_freq 10), systems sharded over the ranks ("strong").

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import math
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
BF16_MFMA_PEAK_TFLOPS = 2500.0         # MI355X_MICROARCH.md: BF16 MFMA, dense (~2.5 PF)
X3_TERMS = 6                           # bf16x3 split: bf16 MFMA products per fp32 product
SPLIT_TERMS = {1: 6, 2: 3}             # 16-bit MFMA products per fp32 product: bf16x3, fp16x2


def segnn_split_prec():
    """The SEGNN split-precision path the library selects (csrc/segnn.hip split_prec)."""
    if os.environ.get("NBX_X3") == "0" or os.environ.get("NBX_SPLIT", "")[:1] == "0":
        return 0
    return 1 if os.environ.get("NBX_SPLIT", "")[:1] in ("x", "1") else 2
FP64_VALU_PEAK_TFLOPS = 78.6           # MI355X spec; no f64 MFMA used by the integrator
SURVEY_GFLOP_PER_STEP = 67.73          # algorithmic work of the reference formulation
COMPULSORY_BYTES_C2 = 8.0e6            # weights 7.79 MB + state I/O ~0.25 MB per C2 step


def initial_states(B, N, seed0):
    from nbody_amd.gravity import GravitySim
    sim = GravitySim(n_balls=N, interaction_strength=2, dt=0.01, softening=0.2, device="cpu")
    loc = np.empty((B, N, 3))
    vel = np.empty((B, N, 3))
    for b in range(B):
        p, v, _ = sim.initial_conditions(seed0 + b)
        loc[b], vel[b] = p, v
    return loc, vel, np.ones((B, N, 1))


def blas_threads():
    return int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))


def timed_region(fn, device, P):
    """barrier + sync on both sides, MAX over ranks."""
    torch.cuda.synchronize(device)
    P.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    out = fn()
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    return out, P.max_over_ranks(elapsed, device)


# ---------------------------------------------------------------- C2 SEGNN (headline)
def cpu_baseline_segnn(loc, vel, mass, steps=1):
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
    threads = blas_threads()
    return {"value": steps / dt, "unit": "steps/s", "cores": threads, "kind": "port",
            "sample": f"{steps} self-feed step(s) of the B={loc.shape[0]} N={loc.shape[1]} batch, numpy fp64 oracle "
                      f"(oracle/segnn.py), BLAS threads={threads}, {dt:.2f} s"}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline_segnn_torch(loc, vel, mass, steps=20):
    """BASELINE.md §3's C2 CPU baseline: the unfused PyTorch CPU restatement of the reference SEGNN
    forward (oracle/segnn_torch.py, fp64 -- the reference's default precision_mode, train-mode
    BatchNorm) driving the self-feed loop of infer_self_feed.py:99-194 for `steps` steps of the full
    B=1024 batch on the host cores (torch threads = OMP_NUM_THREADS)."""
    from oracle import segnn_torch as OT
    from oracle.graph import fc_edge_index
    from oracle.segnn import SEGNNOracle, init_params
    B, N, _ = loc.shape
    om = SEGNNOracle(hidden_features=HIDDEN, num_layers=LAYERS)
    params = {k: torch.tensor(v) for k, v in init_params(om, seed=0).items()}
    threads = blas_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    ei = torch.from_numpy(fc_edge_index(B, N))
    p = torch.from_numpy(loc.reshape(-1, 3)).double()
    v = torch.from_numpy(vel.reshape(-1, 3)).double()
    m = torch.from_numpy(mass.reshape(-1, 1)).double()
    t0 = time.perf_counter()
    with torch.no_grad():
        for _ in range(steps):
            out, stats = OT.forward(om, params, p, v, m, ei, True)
            params.update(stats)
            p, v = p + out[:, :3], out[:, 3:].contiguous()
    dt = time.perf_counter() - t0
    torch.set_num_threads(prev)
    return {"value": steps / dt, "unit": "steps/s", "cores": threads, "kind": "port", "cpu_model": cpu_model(),
            "sample": f"{steps} self-feed steps of the full B={B} N={N} batch, torch fp64 restatement of the reference "
                      f"forward (oracle/segnn_torch.py, train-mode BatchNorm), {threads} threads, {dt:.2f} s"}


def bench_segnn(a, rank, world, device, P):
    import nbody_amd.segnn as S
    from nbody_amd import _lib

    B, N = a.batch or BATCH, NBODY
    torch.manual_seed(0)
    model = S.SEGNN(hidden_features=HIDDEN, num_layers=LAYERS, lmax_h=1,
                    deterministic=a.deterministic_bn).to(device).float().train()
    # BatchNorm statistics: "batch" = per-rank batch statistics (the reference's
    # train-mode rollout on each rank's own B systems), "sync" = batch statistics over every rank's
    # systems (12 RCCL all-reduces of [3][96] fp64 sums per step), "running" = running statistics
    bn_desc = {"batch": "batch statistics per rank (reference train-mode rollout)",
               "sync": "batch statistics over all ranks (SyncBN: 12 all-reduces per step)",
               "running": "running statistics (no batch reduction)"}[a.bn_mode]
    if a.bn_mode == "running":
        model.bn_mode = "running"
    elif a.bn_mode == "sync" and world > 1:
        model.enable_sync_batchnorm(global_batch=B * world)
    loc, vel, mass = initial_states(B, N, rank * B)
    loc_d = torch.tensor(loc, dtype=torch.float32, device=device)
    vel_d = torch.tensor(vel, dtype=torch.float32, device=device)
    mass_d = torch.tensor(mass, dtype=torch.float32, device=device)
    if a.warmup > 0:  # also packs weights / allocates the workspace
        model.rollout(loc_d, vel_d, mass_d, a.warmup + 1)

    def work():
        tp, tv = model.rollout(loc_d, vel_d, mass_d, a.steps + 1)
        final = torch.cat([tp[:, -1], tv[:, -1]], -1).contiguous()
        a.final_states = P.all_gather_shards(final)
        return tp
    tp, elapsed = timed_region(work, device, P)
    finite = bool(torch.isfinite(tp).all().item())
    # diagnostic (outside the timed region): host time to enqueue one rollout of the same length
    # against its device completion, and the device time of the rollout kernels alone (events)
    torch.cuda.synchronize(device)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    h0 = time.perf_counter()
    e0.record()
    model.rollout(loc_d, vel_d, mass_d, a.steps + 1)
    e1.record()
    h1 = time.perf_counter()
    torch.cuda.synchronize(device)
    h2 = time.perf_counter()
    diag = {"host_enqueue_ms": round(1e3 * (h1 - h0), 3), "host_to_done_ms": round(1e3 * (h2 - h0), 3),
            "device_event_ms": round(e0.elapsed_time(e1), 3)}

    # live roofline of the dominant kernel: HIP events around every launch of the
    # fused tensor-product kernels of a few forwards, on the launch stream, split by kind
    V = B * N
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
    # rocprofv3 names of the four timed launch kinds at C2 (csrc/segnn.hip::forward_impl, split_prec):
    # 2 = fp16x2 images (default), 1 = bf16x3 (NBX_SPLIT=x3), 0 = fp32 MFMA (NBX_X3=0)
    prec = segnn_split_prec()
    sk = {2: "StatSKH2", 1: "StatSKX3", 0: "StatSK"}[prec]
    # register-formed dot operands (csrc/segnn.hip msg_dv / upd_dv; fp16x2 only): the schedule types'
    # last parameter
    dv = prec == 2 and os.environ.get("NBX_MSG_DV", "")[:1] != "0"
    udv = prec == 2 and os.environ.get("NBX_UPD_DV", "")[:1] != "0"

    def sk_name(shape, d=0):
        """demangled schedule type: StatSKH2 carries the DV flag as a sixth parameter"""
        return f"nbx::StatSKH2<{shape}, {d}>" if prec == 2 else f"nbx::{sk}<{shape}>"

    msg2 = (f"void nbx::tp_fused_kernel<3, 1, 1, 8, {2 if dv else 3}, {sk_name('6, 6, 3, 3, 0', int(dv))} >"
            "(nbx::TpProb)")
    # (msg_pre's third parameter: the NBX_MP_CHECK hand-off invariant build, 0 unless that switch is set)
    names = [f"void nbx::msg_pre_kernel<{prec}, {3 if prec else 0}, {mp_check_level()}>(nbx::MsgPreProb)",
             msg2,
             f"void nbx::tp16_kernel<3, 1, 2, 1, 8, 3, 1, false, {sk_name('12, 12, 6, 6, 4', int(udv))} >(nbx::TpProb, "
             "nbx::TpProb, int)",
             f"void nbx::tp16_kernel<2, 1, 3, 1, 8, 3, 1, false, "
             f"{sk_name('6, 3, 0, 3, 0', int(udv)) if prec == 2 else 'nbx::StatSK<6, 3, 0, 3, 0>'} >(nbx::TpProb, nbx::TpProb, int)"]
    x3 = prec != 0
    roles = ["message_layer_1: node GEMM + edge combination + gate (flops: the node GEMM)",
             "message_layer_2 + gate + aggregation + BN sums",
             "update_layer_1 + gate (the kind's average includes pre_pool1, once per forward)",
             "update_layer_2 + residual + BN sums"]
    per_kind = {}
    for k in range(4):
        if n_k[k]:
            avg_s = ms_k[k] / n_k[k] / 1e3
            fl = fl_k[k] / n_k[k]
            per_kind[names[k]] = {"role": roles[k], "avg_launch_us": round(avg_s * 1e6, 3),
                                  "gflop_per_launch": round(fl / 1e9, 4), "tflops": round(fl / avg_s / 1e12, 3),
                                  "share_of_forward": round(ms_k[k] / fwd_ms, 3)}
    dom = max(range(4), key=lambda k: ms_k[k])
    dom_avg_s = ms_k[dom] / n_k[dom] / 1e3
    dom_flops = fl_k[dom] / n_k[dom]
    achieved_tflops = dom_flops / dom_avg_s / 1e12
    traffic = pmc_traffic(names[dom], "segnn")
    value = a.steps / elapsed * world
    ms_step = 1e3 * elapsed / a.steps
    # the rocprof duration of the dominant kernel (the same run family as the PMC bytes) and the
    # per-step HBM bytes of the whole step (report the MFMA and the HBM fractions)
    rp_us, rp_src = rocprof_avg_us(names[dom], "segnn")
    pp1 = (f"void nbx::tp16_kernel<3, 1, 2, 1, 8, 3, 1, false, "
           f"{sk_name('6, 6, 3, 3, 2', int(udv)) if prec == 2 else 'nbx::StatSK<6, 6, 3, 3, 2>'} >(nbx::TpProb, nbx::TpProb, int)")
    step_k = [(nm, LAYERS) for nm in names] + [(pp1, 1), ("(anonymous namespace)::rollout_pp2_kernel(", 1)]
    bps, bps_src = step_bytes("segnn", step_k)
    hbm = {"avg_launch_us_rocprof": rp_us, "rocprof_source": rp_src,
           "frac_rocprof": round(dom_flops / (rp_us * 1e-6) / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4) if rp_us else None,
           "hbm_achieved_gbs": round(traffic / (rp_us * 1e-6) / 1e9, 1) if (rp_us and traffic) else None,
           "hbm_frac": round(traffic / (rp_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4) if (rp_us and traffic) else None,
           "bytes_per_step": bps, "bytes_per_step_source": bps_src,
           "compulsory_bytes_per_step": COMPULSORY_BYTES_C2,
           "bytes_over_compulsory": round(bps / COMPULSORY_BYTES_C2, 1) if bps else None,
           "step_hbm_gbs": round(bps / (ms_step * 1e-3) / 1e9, 1) if bps else None,
           "step_hbm_frac": round(bps / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if bps else None,
           "compulsory_hbm_frac": round(COMPULSORY_BYTES_C2 / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)}
    result = {
        "metric": "self-feed rollout steps/sec, SEGNN N=5 batch=1024",
        "value": round(value, 3), "unit": "steps/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(ms_step, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (GravitySim frame-0 initial states, seeded random-init weights)",
        "config": {"workload": "C2: SEGNN lmax_h=1 hidden=192 layers=6, N=5, batch=1024 per GPU, self-feed rollout",
                   "model": "SEGNN", "global_batch": B * world, "seq_len": a.steps, "parallelism": f"dp{world}",
                   "bn_mode": bn_desc, "bn_sums": "fixed order" if a.deterministic_bn else "fp64 atomics"},
        "trajectory_steps_per_s": round(value * B, 1),
        "survey_formulation_tflops": round(value * SURVEY_GFLOP_PER_STEP / 1e3, 3),
        "roofline": {"bound": "mfma", "kernel": names[dom], "achieved": round(achieved_tflops, 3),
                     "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved_tflops / FP32_MFMA_PEAK_TFLOPS, 4), "traffic": traffic,
                     "avg_launch_us": round(dom_avg_s * 1e6, 3), "gflop_per_launch": round(dom_flops / 1e9, 4),
                     # achieved / frac: fp32-accurate GEMM flops against the fp32 MFMA peak; the
                     # split-precision path executes them as X3_TERMS bf16 MFMA products each
                     "mfma_path": {2: "fp16x2 split (fp32-accurate), v_mfma_f32_*_f16",
                                   1: "bf16x3 split (fp32-accurate), v_mfma_f32_*_bf16",
                                   0: "fp32, v_mfma_f32_*_f32"}[prec],
                     # the 16-bit MFMA products actually issued (bf16x3: 6, fp16x2: 3 per fp32 product)
                     "executed_16bit_tflops": round(achieved_tflops * SPLIT_TERMS[prec], 2) if x3 else None,
                     "executed_16bit_frac": (round(achieved_tflops * SPLIT_TERMS[prec] / BF16_MFMA_PEAK_TFLOPS, 4)
                                             if x3 else None),
                     "timing": "achieved / frac: hipExtLaunchKernel start/stop events (kernel execution "
                               "interval, this run); *_rocprof, hbm_*: the committed rocprofv3 profile's average "
                               "duration with its PMC bytes (2 x FETCH_SIZE + WRITE_SIZE)",
                     **hbm,
                     "fused_tp_share_of_forward": round(sum(ms_k) / fwd_ms, 3), "per_kind": per_kind},
        "finite": finite, "rollout_timing": diag,
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        # >= 20 steps of the PyTorch CPU restatement (the reported baseline), beside one
        # step of the numpy oracle (the round-1/2 figure)
        result["cpu_baseline"] = cpu_baseline_segnn_torch(loc, vel, mass, a.cpu_torch_steps)
        result["cpu_baseline"]["numpy_oracle"] = cpu_baseline_segnn(loc, vel, mass, a.cpu_steps)
    return result


def newest_profile(fname):
    """The newest committed profiles/r*/<fname> (the round's HEAD profile), else None."""
    import glob
    c = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", fname)), reverse=True)
    return c[0] if c else None


def mp_check_level():
    """msg_pre's CHK template argument (csrc/msg_pre.hip mp_check_word: NBX_MP_CHECK=1 check, 2 fault injection)."""
    v = os.environ.get("NBX_MP_CHECK", "")
    return int(v) if v in ("1", "2") else 0


def rocprof_avg_us(kernel_name, model):
    """Average duration (us) of `kernel_name` in the newest committed rocprofv3 --stats summary
    (profiles/r*/<model>_kernel_stats.csv, written by scripts/profile_models.sh), else None."""
    import csv
    path = newest_profile(f"{model}_kernel_stats.csv")
    if path is None:
        return None, None
    for r in csv.DictReader(open(path)):
        if r["Name"] == kernel_name:
            return float(r["AverageNs"]) / 1e3, os.path.relpath(path, ROOT)
    return None, os.path.relpath(path, ROOT)


def step_bytes(model, step_kernels):
    """HBM bytes per step from the newest PMC summary: sum over the step's kernels (name or name
    prefix -> launches per step) of their PMC bytes per launch; None if any is missing."""
    path = newest_profile(f"pmc_{model}.json")
    if path is None:
        return None, None
    with open(path) as f:
        kern = json.load(f)["kernels"]
    total = 0
    for name, n in step_kernels:
        hit = [v for k, v in kern.items() if k == name or k.startswith(name)]
        if not hit or hit[0].get("hbm_bytes_per_launch") is None:
            return None, os.path.relpath(path, ROOT)
        total += n * hit[0]["hbm_bytes_per_launch"]
    return total, os.path.relpath(path, ROOT)


def pmc_traffic(kernel_name, model=None):
    """HBM bytes per launch of `kernel_name` from the newest committed PMC summary
    (profiles/r*/pmc_<model>.json, written by scripts/profile_models.sh: 2 x FETCH_SIZE +
    WRITE_SIZE per dispatch, MI355X_MICROARCH.md's gfx950 correction), else None."""
    import glob
    cands = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"pmc_{model}.json")), reverse=True) if model else []
    cands.append(os.path.join(ROOT, "profiles", "pmc_tp_kernels.json"))
    for pmc in cands:
        if os.path.exists(pmc):
            with open(pmc) as f:
                v = json.load(f)["kernels"].get(kernel_name, {}).get("hbm_bytes_per_launch")
            if v is not None:
                return v
    return None


# ---------------------------------------------------------------- C3 PONITA
# rocprofv3 names at C3 (ponita.hip lin_auto: PREC = 2 with the fp16x2 images, the default since r06, 1 with
# the bf16x3 ones (NBX_PO_SPLIT=x3); NT by the image's LDS size; the ConvNext MLP fused into po_ffn_kernel;
# kind 2 (linear_2 alone) only runs on the unfused path)
_PO_PREC = "1" if os.environ.get("NBX_PO_SPLIT", "")[:1] in ("x", "1") else "2"
PONITA_KIND_NAMES = [f"void nbx::lin_kernel<4, 0, 1, {_PO_PREC}>(nbx::LinProb)",
                     f"void (anonymous namespace)::po_ffn_kernel<4, 4, 0, {_PO_PREC}>((anonymous namespace)::FfnProb)",
                     "void nbx::lin_rp_kernel<4, 0, 1>(nbx::LinRpProb)",
                     f"void (anonymous namespace)::po_ffn_kernel<1, 4, 1, {_PO_PREC}>((anonymous namespace)::FfnProb)",
                     "void (anonymous namespace)::po_fiber_ln1_kernel<20, 4, 512>(float const*, float const*, int, "
                     "float const*, float const*, float const*, long, int, int, int, int, float*, double*)"]
PONITA_KIND_ROLES = ["FiberBundleConv spatial kernel GEMM + gather/aggregate epilogue",
                     "ConvNext MLP fused (linear_1 + GELU + linear_2 + layer_scale + residual, hidden in registers)",
                     "ConvNext linear_2 + layer_scale + residual (unfused path only)",
                     "kernel basis MLP (both layers fused, po_ffn_kernel FFN_BASIS)",
                     "fibre conv + bias + LayerNorm"]


def bench_ponita(a, rank, world, device, P):
    from nbody_amd import _lib
    from nbody_amd.ponita import PONITA_NBODY

    B_glob, N = a.batch or 4096, 5
    start, B = P.shard_range(B_glob, rank, world)
    torch.manual_seed(0)
    model = PONITA_NBODY(hidden_dim=128, layers=6, num_ori=20, basis_dim=128, degree=3).to(device)
    if world > 1:   # one calibration from the moments of the whole global batch (conv.py:134-140)
        import torch.distributed as dist
        model.calibration_group = dist.group.WORLD
    loc, vel, mass = initial_states(B, N, start)
    t = lambda x: torch.tensor(x, dtype=torch.float32, device=device)
    loc_d, vel_d, mass_d = t(loc), t(vel), t(mass)
    model.rollout(loc_d, vel_d, mass_d, max(a.warmup, 1) + 1)     # includes the one-time calibration

    def work():
        tp, tv = model.rollout(loc_d, vel_d, mass_d, a.steps + 1)
        a.final_states = P.all_gather_shards(torch.cat([tp[:, -1], tv[:, -1]], -1).contiguous(), B_glob)
        return tp
    tp, elapsed = timed_region(work, device, P)
    finite = bool(torch.isfinite(tp).all().item())

    W = model._weights(device)
    ws = model._workspace(W, B, N, device)
    p32, v32, m32 = loc_d.reshape(-1, 3), vel_d.reshape(-1, 3), mass_d.reshape(-1)
    out = torch.empty(B * N, 6, device=device)
    kms, kn, kfl, kby, tot = (_lib.c_f * 8)(), (_lib.c_i32 * 8)(), (_lib.c_d * 8)(), (_lib.c_d * 8)(), _lib.c_f()
    acc = np.zeros((4, 8))
    fwd = 0.0
    for _ in range(3):
        _lib.check(_lib.lib().nbx_ponita_forward_timed(W, _lib.dev_ptr(p32), _lib.dev_ptr(v32), _lib.dev_ptr(m32),
                                                       B, N, _lib.dev_ptr(out), _lib.dev_ptr(ws), ws.numel(),
                                                       _lib.stream_ptr(device), kms, kn, kfl, kby, tot),
                   "nbx_ponita_forward_timed")
        acc += np.array([list(kms), list(kn), list(kfl), list(kby)])
        fwd += tot.value
    per_kind = {}
    for k in range(5):
        if acc[1, k]:
            s = acc[0, k] / acc[1, k] / 1e3
            per_kind[PONITA_KIND_ROLES[k]] = {
                "kernel": PONITA_KIND_NAMES[k], "avg_launch_us": round(s * 1e6, 2),
                "tflops": round(acc[2, k] / acc[1, k] / s / 1e12, 3),
                "gbs": round(acc[3, k] / acc[1, k] / s / 1e9, 1), "share_of_forward": round(acc[0, k] / fwd, 3)}
    dom = max(range(5), key=lambda k: acc[0, k])
    dom_s = acc[0, dom] / acc[1, dom] / 1e3
    if dom == 4:
        ach = acc[3, dom] / acc[1, dom] / dom_s / 1e9
        roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4)}
    else:
        ach = acc[2, dom] / acc[1, dom] / dom_s / 1e12
        roof = {"bound": "mfma", "achieved": round(ach, 3), "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4)}
    roof.update({"traffic": pmc_traffic(PONITA_KIND_NAMES[dom], "ponita"), "kernel": PONITA_KIND_NAMES[dom],
                 "role": PONITA_KIND_ROLES[dom], "avg_launch_us": round(dom_s * 1e6, 2), "per_kind": per_kind})
    if dom in (0, 1, 3):   # a split-precision GEMM kernel: the 16-bit MFMA products actually issued
        roof.update({"mfma_path": ("fp16x2 split (fp32-accurate), v_mfma_f32_32x32x16_f16" if _PO_PREC == "2" else
                                   "bf16x3 split (fp32-accurate), v_mfma_f32_32x32x16_bf16"),
                     "executed_16bit_frac": round(ach * SPLIT_TERMS[int(_PO_PREC)] / BF16_MFMA_PEAK_TFLOPS, 4)})
    value = a.steps / elapsed
    result = {
        "metric": "self-feed rollout steps/sec, PONITA N=5 batch=4096", "value": round(value, 3), "unit": "steps/s",
        "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(1e3 * elapsed / a.steps, 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (GravitySim frame-0 initial states, seeded random-init weights, calibrated)",
        "config": {"workload": "C3: PONITA hidden=128 layers=6 num_ori=20 basis_dim=128 degree=3, N=5, "
                               f"global batch {B_glob} sharded over {world} GPU(s)", "model": "PONITA",
                   "global_batch": B_glob, "seq_len": a.steps, "parallelism": f"dp{world}"},
        "trajectory_steps_per_s": round(value * B_glob, 1),
        "algorithmic_tflops": round(value * fwd_flops(acc) / 1e12, 3),
        "roofline": roof, "finite": finite}
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline_ponita(model, B_glob)
    return result


def fwd_flops(acc):
    n_fwd = 3
    return acc[2, :5].sum() / n_fwd


def cpu_baseline_ponita(model, B_glob, B_s=64):
    from oracle import ponita as op
    from oracle.graph import fc_edge_index
    params = {k: v.double().cpu().numpy() for k, v in model.state_dict().items()}
    grid = model.model.ori_grid.double().cpu().numpy()
    loc, vel, mass = initial_states(B_s, 5, 0)
    pos, v, m = loc.reshape(-1, 3), vel.reshape(-1, 3), mass.reshape(-1, 1)
    ei = fc_edge_index(B_s, 5)
    t0 = time.perf_counter()
    op.forward(params, m, v[:, None, :], ei, pos[ei[0]] - pos[ei[1]], grid, 6)
    dt = time.perf_counter() - t0
    threads = blas_threads()
    return {"value": 1.0 / (dt * B_glob / B_s), "unit": "steps/s", "cores": threads, "kind": "port",
            "sample": f"1 forward of B={B_s} systems with the numpy fp64 oracle (oracle/ponita.py), {dt:.2f} s, "
                      f"scaled x{B_glob // B_s} to the B={B_glob} batch; BLAS threads={threads}"}


# ---------------------------------------------------------------- C1 EGNN-MC
def bench_egnn(a, rank, world, device, P):
    from nbody_amd.egnn_mc import EGNNMultiChannel
    B, N = a.batch or 64, 5
    torch.manual_seed(0)
    model = EGNNMultiChannel(node_input_dim=2, edge_attr_dim=4, hidden_node_dim=128, hidden_edge_dim=128,
                             hidden_coord_dim=128, num_layers=6, target_names=("pos_dt", "vel"), norm_diff=True,
                             tanh=True, device=device)
    loc, vel, mass = initial_states(B, N, rank * B)
    t = lambda x: torch.tensor(x, dtype=torch.float32, device=device)
    loc_d, vel_d, mass_d = t(loc), t(vel), t(mass)
    model.rollout(loc_d, vel_d, mass_d, max(a.warmup, 1) + 1)

    def work():
        tp, tv = model.rollout(loc_d, vel_d, mass_d, a.steps + 1)
        a.final_states = P.all_gather_shards(torch.cat([tp[:, -1], tv[:, -1]], -1).contiguous())
        return tp
    tp, elapsed = timed_region(work, device, P)
    value = a.steps / elapsed * world
    result = {
        "metric": "self-feed rollout steps/sec, EGNN-MC N=5 batch=64", "value": round(value, 3), "unit": "steps/s",
        "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(1e3 * elapsed / a.steps, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (GravitySim frame-0 initial states, seeded random-init weights)",
        "config": {"workload": "C1: EGNN-MC 6 x 128, norm_diff, tanh, N=5, batch 64 per GPU", "model": "EGNN-MC",
                   "global_batch": B * world, "seq_len": a.steps, "parallelism": f"dp{world}"},
        "roofline": {"bound": "latency", "achieved": None, "peak": None, "unit": None, "frac": None, "traffic": None,
                     "kernel": "egnn_persist_kernel<128>: one workgroup per system runs the whole rollout",
                     "note": "C1 is latency bound (SURVEY §8d): 64 systems = 64 workgroups, each a serial chain of "
                             "~30 dependent block GEMM / reduction phases per layer on 20 edges; one launch per "
                             "rollout (was ~60 launches per step)"},
        "finite": bool(torch.isfinite(tp).all().item())}
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        from oracle.rollout import egnn_mc_step, rollout
        params = {k: v.double().cpu().numpy() for k, v in model.state_dict().items()}
        steps = 20
        t0 = time.perf_counter()
        rollout(egnn_mc_step(params, 6), loc, vel, np.zeros_like(loc), mass, steps + 1)
        dt = time.perf_counter() - t0
        result["cpu_baseline"] = {"value": steps / dt, "unit": "steps/s", "cores": blas_threads(), "kind": "port",
                                  "sample": f"{steps} self-feed steps of the B={B} batch, numpy fp64 oracle "
                                            f"(oracle/egnn_mc.py), {dt:.2f} s"}
    return result


# ---------------------------------------------------------------- C1-shaped EGNN-MC training step
def bench_egnn_train(a, rank, world, device, P):
    """one training step of the reference trainer (trainer.py:233-358, standard
    precision): zero_grad, native forward (activations kept), MSE loss, loss.backward() -> native
    backward (csrc/egnn_train.hip), gradient all-reduce over ranks (data parallel, RCCL), clip to
    norm 1, AdamW step + LambdaLR (trainer.py:170-194).  C1 widths (6 x 128), N=5, batch 64 per
    rank ("weak")."""
    from nbody_amd.egnn_mc import EGNNMultiChannel
    B, N = a.batch or 64, 5
    torch.manual_seed(0)
    model = EGNNMultiChannel(node_input_dim=2, edge_attr_dim=4, hidden_node_dim=128, hidden_edge_dim=128,
                             hidden_coord_dim=128, num_layers=6, target_names=("pos_dt", "vel"), norm_diff=True,
                             tanh=True, device=device)
    loc, vel, mass = initial_states(B, N, rank * B)
    rng = np.random.default_rng(100 + rank)

    class _G:
        pass
    from nbody_amd.graph import fc_edge_index
    g = _G()
    t = lambda x: torch.tensor(x, dtype=torch.float32, device=device)
    g.pos, g.vel, g.mass = t(loc.reshape(-1, 3)), t(vel.reshape(-1, 3)), t(mass.reshape(-1, 1))
    g.edge_index = fc_edge_index(B, N, device)
    g.nbx_system_size = N
    target = t(rng.standard_normal((B * N, 6)) * 0.1)
    # Trainer.create_optimizer / create_lr_scheduler (trainer.py:170-194): AdamW(weight_decay 1e-8,
    # betas (0.9, 0.98), eps 1e-9) under the LambdaLR warmup schedule; the update as one fused launch
    # one HIP graph per step on one GPU; with several ranks the gradient all-reduce (RCCL) would be
    # recorded inside the graph, a path not yet validated on hardware: eager until it is
    graph = not a.eager and world == 1
    opt = torch.optim.AdamW(model.parameters(), lr=1.0, weight_decay=1e-8, betas=(0.9, 0.98), eps=1e-9,
                            fused=True, capturable=graph)
    sched = torch.optim.lr_scheduler.LambdaLR(
        opt, lambda s: 128 ** -0.5 * min(max(s, 1) ** -0.5, max(s, 1) * 1000 ** -1.5))
    if graph:
        # the scheduler keeps float base lrs and writes each step's lr into this device tensor
        # (LRScheduler fills tensor lrs in place), which the captured fused AdamW reads
        for grp in opt.param_groups:
            grp["lr"] = torch.tensor(float(grp["lr"]), dtype=torch.float32, device=device)
    params = list(model.parameters())

    def step_body():
        # (captured too: backward then allocates the gradients in the graph's pool, so replays
        # rewrite the same buffers and no per-parameter fill / accumulate launches are recorded)
        opt.zero_grad(set_to_none=True)
        loss = torch.nn.functional.mse_loss(model(g), target)
        loss.backward()
        P.allreduce_gradients(params)   # data parallel over RCCL (one bucket at C1); no-op on one rank
        torch.nn.utils.clip_grad_norm_(params, 1.0, foreach=True)
        opt.step()
        return loss

    if graph:
        # HIP graph of the whole step (native forward / backward launches, clip, fused AdamW): one
        # replay per step instead of ~1 ms of per-step host work for 60 parameter tensors
        side = torch.cuda.Stream(device)
        side.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(side):
            for _ in range(max(a.warmup, 3)):
                step_body()
                sched.step()
        torch.cuda.current_stream(device).wait_stream(side)
        cg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(cg):
            static_loss = step_body()

        def train_step():
            cg.replay()
            sched.step()
            model.invalidate_weights()   # the replay's AdamW updated the parameters in place
            return static_loss
    else:
        def train_step():
            loss = step_body()
            sched.step()
            return loss

    for _ in range(max(a.warmup, 1)):
        train_step()

    def work():
        for _ in range(a.steps):
            loss = train_step()
        return loss
    loss, elapsed = timed_region(work, device, P)
    value = a.steps / elapsed * world
    result = {
        "metric": "EGNN-MC training steps/sec (C1 widths, forward + backward + AdamW)", "value": round(value, 3),
        "unit": "train steps/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(1e3 * elapsed / a.steps, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (GravitySim frame-0 initial states, random targets, seeded random-init weights)",
        "config": {"workload": "SURVEY 8(f)4: EGNN-MC 6 x 128 training step, N=5, batch 64 per GPU, MSE loss, "
                               "grad-norm clip 1, AdamW + LambdaLR (trainer.py:170-194)", "model": "EGNN-MC", "global_batch": B * world,
                   "seq_len": a.steps, "parallelism": f"dp{world}",
                   "execution": "one HIP graph replay per step (forward, backward, clip, fused AdamW)" if graph
                                else "eager"},
        "roofline": {"bound": "latency", "achieved": None, "peak": None, "unit": None, "frac": None, "traffic": None,
                     "kernel": "egnn_train_fwd_kernel / egnn_train_bwd_kernel: one workgroup per system",
                     "note": "64 systems = 64 workgroups of 20-edge fp32 reductions: latency bound like C1"},
        "loss": float(loss.item()), "finite": bool(math.isfinite(float(loss.item())))}
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        from oracle import egnn_mc_torch as OT
        Pc = {k: v.detach().double().cpu().clone().requires_grad_(True) for k, v in model.named_parameters()}
        optc = torch.optim.AdamW(list(Pc.values()), lr=1e-4, weight_decay=1e-8, betas=(0.9, 0.98), eps=1e-9)
        pc, vc, mc = (torch.from_numpy(x.reshape(-1, w)).double() for x, w in ((loc, 3), (vel, 3), (mass, 1)))
        tc = target.double().cpu()
        steps = 10
        t0 = time.perf_counter()
        for _ in range(steps):
            optc.zero_grad()
            lc = torch.nn.functional.mse_loss(OT.forward(Pc, pc, vc, mc, B, N, 6), tc)
            lc.backward()
            torch.nn.utils.clip_grad_norm_(list(Pc.values()), 1.0)
            optc.step()
        dt = time.perf_counter() - t0
        result["cpu_baseline"] = {"value": steps / dt, "unit": "train steps/s", "cores": torch.get_num_threads(),
                                  "kind": "port", "sample": f"{steps} training steps of the B={B} batch, torch fp64 "
                                                            f"autograd restatement (oracle/egnn_mc_torch.py), {dt:.2f} s"}
    return result


# ---------------------------------------------------------------- SEGNN training step
def train_loop(a, world, device, P, model, forward, target, model_size):
    """The reference trainer's step (trainer.py:170-194,233-358): zero_grad, forward, MSE loss,
    loss.backward(), gradient all-reduce over ranks (RCCL), clip to norm 1, AdamW (weight decay 1e-8,
    betas (0.9, 0.98), eps 1e-9) + LambdaLR (factor 1, warmup 1000, model_size^-0.5).  One eager step
    first (it also performs any one-time calibration) with every nbx_gemm_f32 launch event-timed for
    the roofline; on one GPU the step is then captured as one HIP graph (--eager: uncaptured).
    Returns (last loss, timed seconds, (gemm ms, gemm flops, gemm launches) of one step, graph?)."""
    import nbody_amd.segnn_train as ST
    graph = not a.eager and world == 1
    opt = torch.optim.AdamW(model.parameters(), lr=1.0, weight_decay=1e-8, betas=(0.9, 0.98), eps=1e-9,
                            fused=True, capturable=graph)
    sched = torch.optim.lr_scheduler.LambdaLR(
        opt, lambda s: model_size ** -0.5 * min(max(s, 1) ** -0.5, max(s, 1) * 1000 ** -1.5))
    if graph:
        for grp in opt.param_groups:
            grp["lr"] = torch.tensor(float(grp["lr"]), dtype=torch.float32, device=device)
    params = list(model.parameters())

    def step_body():
        opt.zero_grad(set_to_none=True)
        loss = torch.nn.functional.mse_loss(forward(), target)
        loss.backward()
        P.allreduce_gradients(params)
        torch.nn.utils.clip_grad_norm_(params, 1.0, foreach=True)
        opt.step()
        return loss

    # roofline: every GEMM launch of one eager step, event-timed on the launch stream
    ST.gemm_timer = []
    step_body()
    torch.cuda.synchronize(device)
    gemm = (sum(e0.elapsed_time(e1) for e0, e1, _ in ST.gemm_timer), sum(f for _, _, f in ST.gemm_timer),
            len(ST.gemm_timer))
    ST.gemm_timer = None
    sched.step()
    if graph:
        side = torch.cuda.Stream(device)
        side.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(side):
            for _ in range(max(a.warmup, 3)):
                step_body()
                sched.step()
        torch.cuda.current_stream(device).wait_stream(side)
        cg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(cg):
            static_loss = step_body()

        def train_step():
            cg.replay()
            sched.step()
            return static_loss
    else:
        def train_step():
            loss = step_body()
            sched.step()
            return loss

    for _ in range(max(a.warmup, 1)):
        train_step()

    def work():
        for _ in range(a.steps):
            loss = train_step()
        return loss
    loss, elapsed = timed_region(work, device, P)
    return loss, elapsed, gemm, graph


def bench_segnn_train(a, rank, world, device, P):
    """one SEGNN training step of the reference trainer (trainer.py:233-358) at C2
    widths (hidden 192, lmax 1, 6 layers, N=5) on the reference's training batch (config.yaml
    dataloaders batch_size 64 systems per rank, "weak"): zero_grad, train-mode forward on the native
    training operators (segnn_train.py / csrc/segnn_train.hip), MSE loss, loss.backward() through the
    native backward, gradient all-reduce over ranks (RCCL), clip to norm 1, AdamW + LambdaLR
    (trainer.py:170-194).  On one GPU the whole step is one HIP graph replay (--eager: uncaptured)."""
    import nbody_amd.segnn as S
    import nbody_amd.segnn_train as ST
    from nbody_amd.graph import fc_edge_index
    B, N = a.batch or 64, NBODY
    torch.manual_seed(0)
    model = S.SEGNN(hidden_features=HIDDEN, num_layers=LAYERS).to(device).train()
    loc, vel, mass = initial_states(B, N, rank * B)
    rng = np.random.default_rng(100 + rank)

    class _G:
        pass
    g = _G()
    t = lambda x: torch.tensor(x, dtype=torch.float32, device=device)
    g.pos, g.vel, g.mass = t(loc.reshape(-1, 3)), t(vel.reshape(-1, 3)), t(mass.reshape(-1, 1))
    g.edge_index = fc_edge_index(B, N, device)
    g.nbx_system_size = N
    target = t(rng.standard_normal((B * N, 6)) * 0.1)
    loss, elapsed, gemm, graph = train_loop(a, world, device, P, model, lambda: model(g), target, HIDDEN)
    model.invalidate_weights()   # the replays' AdamW updated the parameters in place
    value = a.steps / elapsed * world
    gemm_ms, gemm_flops, n_gemm = gemm
    ach = gemm_flops / (gemm_ms * 1e-3) / 1e12 if gemm_ms > 0 else None
    result = {
        "metric": "SEGNN training steps/sec (C2 widths, forward + backward + AdamW)", "value": round(value, 3),
        "unit": "train steps/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(1e3 * elapsed / a.steps, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (GravitySim frame-0 initial states, random targets, seeded random-init weights)",
        "config": {"workload": "SURVEY 8(f)4: SEGNN lmax_h=1 hidden 192, 6 layers training step, N=5, batch 64 per "
                               "GPU (config.yaml batch_size), train-mode BatchNorm, MSE loss, grad-norm clip 1, "
                               "AdamW + LambdaLR (trainer.py:170-194)", "model": "SEGNN", "global_batch": B * world,
                   "seq_len": a.steps, "parallelism": f"dp{world}",
                   "execution": "one HIP graph replay per step (forward, backward, clip, fused AdamW)" if graph
                                else "eager"},
        "roofline": {"bound": "mfma", "kernel": "gemm_f32_batched_kernel (nbx_gemm_f32_batched: every tensor-product "
                                               "GEMM of the forward and backward, grouped per tensor product)",
                     "achieved": round(ach, 3) if ach else None, "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4) if ach else None,
                     "traffic": pmc_traffic("(anonymous namespace)::gemm_f32_batched_kernel((anonymous namespace)::"
                                            "GemmBatch)", "segnn_train"),
                     "avg_launch_us": round(1e3 * gemm_ms / max(n_gemm, 1), 3), "launches_per_step": n_gemm,
                     "gflop_per_step": round(gemm_flops / 1e9, 4),
                     "timing": "torch.cuda.Event pairs around every GEMM launch of one eager step, launch stream",
                     "note": "B=64 training batch: GEMMs of 320-1280 rows, latency-bound"},
        "loss": float(loss.item()), "finite": bool(math.isfinite(float(loss.item())))}
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        from oracle import segnn_torch as OT
        from oracle.graph import fc_edge_index as oei
        from oracle.segnn import SEGNNOracle
        om = SEGNNOracle(hidden_features=HIDDEN, num_layers=LAYERS)
        Pc = {k: v.detach().double().cpu().clone().requires_grad_("running" not in k)
              for k, v in model.state_dict().items() if "output_mask" not in k}
        optc = torch.optim.AdamW([v for v in Pc.values() if v.requires_grad], lr=1e-4, weight_decay=1e-8,
                                 betas=(0.9, 0.98), eps=1e-9)
        tt = lambda x, w: torch.from_numpy(x.reshape(-1, w)).double()
        pc, vc, mc = tt(loc, 3), tt(vel, 3), tt(mass, 1)
        ei = torch.from_numpy(oei(B, N))
        tc = target.double().cpu()
        steps = max(1, a.cpu_steps)
        t0 = time.perf_counter()
        for _ in range(steps):
            optc.zero_grad()
            lc = torch.nn.functional.mse_loss(OT.forward(om, Pc, pc, vc, mc, ei, True)[0], tc)
            lc.backward()
            torch.nn.utils.clip_grad_norm_([v for v in Pc.values() if v.requires_grad], 1.0)
            optc.step()
        dt = time.perf_counter() - t0
        result["cpu_baseline"] = {"value": steps / dt, "unit": "train steps/s", "cores": torch.get_num_threads(),
                                  "kind": "port", "sample": f"{steps} training step(s) of the B={B} batch, torch fp64 "
                                                            f"autograd restatement (oracle/segnn_torch.py), {dt:.2f} s"}
    return result


PONITA_TRAIN = dict(hidden_dim=128, layers=8, num_ori=20, basis_dim=128)   # config.yaml models.ponita


def bench_ponita_train(a, rank, world, device, P):
    """one PONITA training step of the reference trainer (trainer.py:233-358) at the
    reference's PONITA training configuration (config.yaml: hidden 128, 8 layers, 20 orientations,
    basis 128, batch_size 64 systems of N=5 per rank, num_neighbors 4 = fully connected; "weak"):
    zero_grad, forward on the native training operators (ponita_train.py / csrc/ponita_train.hip +
    nbx_gemm_f32), MSE loss, loss.backward() through the native backward, gradient all-reduce over
    ranks, clip, AdamW + LambdaLR.  The one-time FiberBundleConv calibration happens in the first
    (untimed) step's no-grad forward, as the reference's train.py:49-77 dummy forward."""
    import nbody_amd.ponita as PO
    B, N = a.batch or 64, NBODY
    torch.manual_seed(0)
    model = PO.PONITA_NBODY(**PONITA_TRAIN).to(device).train()
    model.model.materialize()
    loc, vel, mass = initial_states(B, N, rank * B)
    rng = np.random.default_rng(200 + rank)
    from nbody_amd.graph import build_graph_with_knn

    class _G:
        pass
    g = _G()
    t = lambda x: torch.tensor(x, dtype=torch.float32, device=device)
    g.pos, g.vec, g.x = t(loc.reshape(-1, 3)), t(vel.reshape(-1, 1, 3)), t(mass.reshape(-1, 1))
    g.edge_index = build_graph_with_knn(g.pos, B, N, device, N - 1)
    g.nbx_system_size = N        # no host synchronisation inside the captured step
    target = t(rng.standard_normal((B * N, 6)) * 0.1)
    loss, elapsed, gemm, graph = train_loop(a, world, device, P, model, lambda: model(g), target,
                                            model.get_model_size())
    gemm_ms, gemm_flops, n_gemm = gemm
    value = a.steps / elapsed * world
    ach = gemm_flops / (gemm_ms * 1e-3) / 1e12 if gemm_ms > 0 else None
    result = {
        "metric": "PONITA training steps/sec (reference training config, forward + backward + AdamW)",
        "value": round(value, 3), "unit": "train steps/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(1e3 * elapsed / a.steps, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (GravitySim frame-0 initial states, random targets, seeded random-init weights)",
        "config": {"workload": "SURVEY 8(f)4: PONITA hidden 128, 8 layers, 20 orientations, basis 128 training "
                               "step, N=5, batch 64 per GPU (config.yaml), MSE loss, grad-norm clip 1, AdamW + "
                               "LambdaLR (trainer.py:170-194)", "model": "PONITA", "global_batch": B * world,
                   "seq_len": a.steps, "parallelism": f"dp{world}",
                   "execution": "one HIP graph replay per step (forward, backward, clip, fused AdamW)" if graph
                                else "eager"},
        "roofline": {"bound": "mfma", "kernel": "gemm_f32_kernel (nbx_gemm_f32: every nn.Linear of the forward and "
                                               "backward)",
                     "achieved": round(ach, 3) if ach else None, "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4) if ach else None, "traffic": None,
                     "avg_launch_us": round(1e3 * gemm_ms / max(n_gemm, 1), 3), "launches_per_step": n_gemm,
                     "gflop_per_step": round(gemm_flops / 1e9, 4),
                     "timing": "torch.cuda.Event pairs around every GEMM launch of one eager step, launch stream"},
        "loss": float(loss.item()), "finite": bool(math.isfinite(float(loss.item())))}
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        from oracle import ponita_torch as OT
        Pc = {k: v.detach().double().cpu().clone().requires_grad_(not (k.endswith("callibrated") or
                                                                       k.endswith("ori_grid")))
              for k, v in model.state_dict().items()}
        learn = [v for v in Pc.values() if v.requires_grad]
        optc = torch.optim.AdamW(learn, lr=1e-4, weight_decay=1e-8, betas=(0.9, 0.98), eps=1e-9)
        pc = torch.from_numpy(loc.reshape(-1, 3))
        vc, mc = torch.from_numpy(vel.reshape(-1, 1, 3)), torch.from_numpy(mass.reshape(-1, 1))
        ei = g.edge_index.cpu()
        grid = Pc["model.ori_grid"]
        tc = target.double().cpu()
        steps = max(1, a.cpu_steps)
        t0 = time.perf_counter()
        for _ in range(steps):
            optc.zero_grad()
            lc = torch.nn.functional.mse_loss(
                OT.forward(Pc, mc, vc, ei, pc[ei[0]] - pc[ei[1]], grid, PONITA_TRAIN["layers"]), tc)
            lc.backward()
            torch.nn.utils.clip_grad_norm_(learn, 1.0)
            optc.step()
        dt = time.perf_counter() - t0
        result["cpu_baseline"] = {"value": steps / dt, "unit": "train steps/s", "cores": torch.get_num_threads(),
                                  "kind": "port", "sample": f"{steps} training step(s) of the B={B} batch, torch fp64 "
                                                            f"autograd restatement (oracle/ponita_torch.py; the "
                                                            f"reference trains PONITA in float64), {dt:.2f} s"}
    return result


# ---------------------------------------------------------------- C4 EquiformerV2
EQV2_C4 = dict(num_layers=4, attn_hidden_channels=64, sphere_channels=64, num_heads=4, attn_alpha_channels=8,
               attn_value_channels=4, ffn_hidden_channels=64, lmax_list=[2], mmax_list=[1], grid_resolution=None,
               edge_channels=64, use_atom_edge_embedding=True, share_atom_edge_embedding=False,
               distance_function="projection", num_distance_basis=64, attn_activation="scaled_silu",
               use_s2_act_attn=False, ffn_activation="scaled_silu", max_neighbors=5, max_radius=4096.0)
EQV2_KINDS = ["radial hidden layers (per-edge layer + GEMM with LayerNorm/SiLU epilogue)",
              "radial output GEMM + rotated-message epilogue (A0/A1)", "SO(2) conv 1, m=0 GEMM",
              "SO(2) conv 1, m=1 GEMM", "separable S2 activation + attention logits", "SO(2) conv 2 GEMMs",
              "node kernels (softmax, inverse rotation, proj, FFN, norms)", "edge frame + edge-degree embedding"]
# rocprofv3 names of the one-launch GEMM kinds at C4 (eqv2.hip gemm_rp: row-panel split-precision GEMM, all
# output columns per workgroup; 288 = 32 alpha + 4 x 64 hidden m=0 outputs -> 9 tiles, 4 x 64 m=1 outputs -> 8;
# PREC 2 on the fp16x2 images, the default since r06, 1 on the bf16x3 ones with NBX_EQ_SPLIT=x3)
_EQ_PREC = "1" if os.environ.get("NBX_EQ_SPLIT", "")[:1] in ("x", "1") else "2"
EQV2_GEMM_NAMES = {2: f"void nbx::lin_rp_kernel<9, 0, {_EQ_PREC}>(nbx::LinRpProb)",
                   3: f"void nbx::lin_rp_kernel<8, 0, {_EQ_PREC}>(nbx::LinRpProb)"}


def bench_eqv2(a, rank, world, device, P):
    from nbody_amd import _lib
    from nbody_amd.equiformer_v2 import EquiformerV2_nbody
    B, N = a.batch or 256, 20
    torch.manual_seed(0)
    model = EquiformerV2_nbody(**EQV2_C4).to(device).eval()
    loc, vel, mass = initial_states(B, N, rank * B)
    t = lambda x: torch.tensor(x, dtype=torch.float32, device=device)
    loc_d, vel_d, mass_d = t(loc), t(vel), t(mass)
    model.rollout(loc_d, vel_d, mass_d, max(a.warmup, 1) + 1, seed=1)

    def work():
        tp, tv = model.rollout(loc_d, vel_d, mass_d, a.steps + 1, seed=2)
        a.final_states = P.all_gather_shards(torch.cat([tp[:, -1], tv[:, -1]], -1).contiguous())
        return tp
    tp, elapsed = timed_region(work, device, P)
    finite = bool(torch.isfinite(tp).all().item())

    W = model._weights(device)
    ws = model._workspace(W, B, N, device)
    p32, v32, m32 = loc_d.reshape(-1, 3), vel_d.reshape(-1, 3), mass_d.reshape(-1)
    out = torch.empty(B * N, 6, device=device)
    kms, kn, kfl, kby, tot = (_lib.c_f * 8)(), (_lib.c_i32 * 8)(), (_lib.c_d * 8)(), (_lib.c_d * 8)(), _lib.c_f()
    acc = np.zeros((4, 8))
    fwd, reps = 0.0, 3
    for _ in range(reps):
        _lib.check(_lib.lib().nbx_eqv2_forward_timed(W, _lib.dev_ptr(p32), _lib.dev_ptr(v32), _lib.dev_ptr(m32), B, N,
                                                     None, 7, _lib.dev_ptr(out), _lib.dev_ptr(ws), ws.numel(),
                                                     _lib.stream_ptr(device), kms, kn, kfl, kby, tot),
                   "nbx_eqv2_forward_timed")
        acc += np.array([list(kms), list(kn), list(kfl), list(kby)])
        fwd += tot.value
    per_kind = {}
    for k in range(8):
        if acc[1, k]:
            sec = acc[0, k] / 1e3
            per_kind[EQV2_KINDS[k]] = {"avg_group_us": round(sec / acc[1, k] * 1e6, 2),
                                       "tflops": round(acc[2, k] / sec / 1e12, 3),
                                       "gbs": round(acc[3, k] / sec / 1e9, 1), "share_of_forward": round(acc[0, k] / fwd, 3)}
    # dominant kernel: the larger of the two SO(2) conv 1 row-panel GEMMs (one launch per attention block each)
    dom = max(EQV2_GEMM_NAMES, key=lambda k: acc[0, k])
    g_avg_s = acc[0, dom] / acc[1, dom] / 1e3
    ach = acc[2, dom] / (acc[0, dom] / 1e3) / 1e12
    gemm_ms = acc[0, 2] + acc[0, 3] + acc[0, 5]
    roof = {"bound": "mfma", "kernel": EQV2_GEMM_NAMES[dom], "role": EQV2_KINDS[dom], "achieved": round(ach, 3),
            "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4),
            "traffic": pmc_traffic(EQV2_GEMM_NAMES[dom], "eqv2"), "avg_launch_us": round(g_avg_s * 1e6, 2),
            "gflop_per_launch": round(acc[2, dom] / acc[1, dom] / 1e9, 4),
            "algorithmic_mb_per_launch": round(acc[3, dom] / acc[1, dom] / 1e6, 3),
            "mfma_path": ("fp16x2 split (fp32-accurate), v_mfma_f32_32x32x16_f16" if _EQ_PREC == "2" else
                          "bf16x3 split (fp32-accurate), v_mfma_f32_32x32x16_bf16"),
            # the 16-bit MFMA products actually issued (bf16x3: 6, fp16x2: 3 per fp32 product)
            "executed_16bit_tflops": round(ach * SPLIT_TERMS[int(_EQ_PREC)], 2),
            "executed_16bit_frac": round(ach * SPLIT_TERMS[int(_EQ_PREC)] / BF16_MFMA_PEAK_TFLOPS, 4),
            "timing": "HIP event pairs around each launch group on the launch stream",
            "gemm_share_of_forward": round(gemm_ms / fwd, 3), "per_kind": per_kind}
    value = a.steps / elapsed * world
    result = {
        "metric": "self-feed rollout steps/sec, EquiformerV2 N=20 batch=256", "value": round(value, 3),
        "unit": "steps/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(1e3 * elapsed / a.steps, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (GravitySim frame-0 initial states N=20, seeded random-init weights, device-hash edge gauges)",
        "config": {"workload": "C4: EquiformerV2 4 layers, sphere 64, attn hidden 64, 4 heads (alpha 8, value 4), "
                               "ffn 64, lmax [2], mmax [1], edge channels 64, N=20, batch 256 per GPU",
                   "model": "EquiformerV2", "global_batch": B * world, "seq_len": a.steps, "parallelism": f"dp{world}"},
        "trajectory_steps_per_s": round(value * B, 1),
        "algorithmic_tflops": round(value / world * acc[2].sum() / reps / 1e12, 3),
        "roofline": roof, "finite": finite}
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline_eqv2(model, B)
    return result


def bench_eqv2_train(a, rank, world, device, P):
    """one EquiformerV2 training step of the reference trainer (trainer.py:233-358) at
    the reference's EquiformerV2 training configuration (config.yaml: the C4 widths, batch_size 64
    systems of N=5 per rank; the constructor's alpha_drop 0.1 / drop_path_rate 0.05 in train mode;
    "weak"): zero_grad, forward on the native training operators (eqv2_train.py /
    csrc/eqv2_train.hip + nbx_gemm_f32), MSE loss, loss.backward(), gradient all-reduce over ranks, clip,
    AdamW + LambdaLR."""
    from nbody_amd.equiformer_v2 import EquiformerV2_nbody
    B, N = a.batch or 64, NBODY
    torch.manual_seed(0)
    model = EquiformerV2_nbody(**EQV2_C4).to(device).train()
    loc, vel, mass = initial_states(B, N, rank * B)
    rng = np.random.default_rng(300 + rank)
    t = lambda x: torch.tensor(x, dtype=torch.float32, device=device)
    pos, vv, q = t(loc.reshape(-1, 3)), t(vel.reshape(-1, 3)), t(mass.reshape(-1, 1))
    batch = torch.arange(B, device=device).repeat_interleave(N)
    gauge = t(rng.uniform(0, 1, (B * N * (N - 1), 3)))      # fixed gauges: no host-side counter in the graph
    data = (pos, vv, torch.zeros_like(pos), q, pos)
    target = t(rng.standard_normal((B * N, 6)) * 0.1)
    import nbody_amd.eqv2_train as ET
    fwd = lambda: ET.train_forward(model, pos, vv, q.reshape(-1), B, N, gauge, 0)
    model(data, batch, gauge=gauge)          # the module's own entry point once (grad mode -> eqv2_train)
    loss, elapsed, gemm, graph = train_loop(a, world, device, P, model, fwd, target, model.get_model_size())
    gemm_ms, gemm_flops, n_gemm = gemm
    value = a.steps / elapsed * world
    ach = gemm_flops / (gemm_ms * 1e-3) / 1e12 if gemm_ms > 0 else None
    result = {
        "metric": "EquiformerV2 training steps/sec (reference training config, forward + backward + AdamW)",
        "value": round(value, 3), "unit": "train steps/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(1e3 * elapsed / a.steps, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (GravitySim frame-0 initial states, random targets and gauges, seeded random-init weights)",
        "config": {"workload": "SURVEY 8(f)4: EquiformerV2 C4 widths (4 layers, sphere 64, lmax 2 / mmax 1) training "
                               "step, N=5, batch 64 per GPU (config.yaml), alpha dropout 0.1 + drop path 0.05, MSE "
                               "loss, grad-norm clip 1, AdamW + LambdaLR (trainer.py:170-194)",
                   "model": "EquiformerV2", "global_batch": B * world, "seq_len": a.steps,
                   "parallelism": f"dp{world}",
                   "execution": "one HIP graph replay per step (forward, backward, clip, fused AdamW)" if graph
                                else "eager"},
        "roofline": {"bound": "mfma", "kernel": "gemm_f32 / gemm_f32_batched kernels (nbx_gemm_f32 / _batched / "
                                               "_grouped: every linear layer, SO3_LinearV2 and SO2_Convolution of "
                                               "the forward and backward, each grouped launch timed whole)",
                     "achieved": round(ach, 3) if ach else None, "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4) if ach else None, "traffic": None,
                     "avg_launch_us": round(1e3 * gemm_ms / max(n_gemm, 1), 3), "launches_per_step": n_gemm,
                     "gflop_per_step": round(gemm_flops / 1e9, 4),
                     "timing": "torch.cuda.Event pairs around every GEMM launch of one eager step, launch stream"},
        "loss": float(loss.item()), "finite": bool(math.isfinite(float(loss.item())))}
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        from oracle import equiformer_v2 as EQ
        Pc = {k: v.detach().double().cpu().clone().requires_grad_() for k, v in model.named_parameters()}
        optc = torch.optim.AdamW(list(Pc.values()), lr=1e-4, weight_decay=1e-8, betas=(0.9, 0.98), eps=1e-9)
        gc, tc = gauge.double().cpu(), target.double().cpu()
        steps = max(1, a.cpu_steps)
        t0 = time.perf_counter()
        for _ in range(steps):
            optc.zero_grad()
            lc = torch.nn.functional.mse_loss(EQ.forward(EQV2_C4, Pc, loc, vel, mass, B, N, gc), tc)
            lc.backward()
            torch.nn.utils.clip_grad_norm_(list(Pc.values()), 1.0)
            optc.step()
        dt = time.perf_counter() - t0
        result["cpu_baseline"] = {"value": steps / dt, "unit": "train steps/s", "cores": torch.get_num_threads(),
                                  "kind": "port", "sample": f"{steps} training step(s) of the B={B} batch, torch fp64 "
                                                            f"autograd of oracle/equiformer_v2.py (no dropout), "
                                                            f"{dt:.2f} s"}
    return result


def bench_eqv2_l6(a, rank, world, device, P):
    """The reference constructor's default degrees (lmax_list [6], mmax_list [2],
    equiformer_v2_nbody.py:122-123) at the C4 widths: self-feed rollout on the composed native path
    (eqv2_train.py on csrc/eqv2_general.hip + the generic operators; no fused kernels exist for
    these degrees), N=20, batch 64 per GPU, device-hash edge gauges."""
    from nbody_amd.equiformer_v2 import EquiformerV2_nbody
    B, N = a.batch or 64, 20
    cfg = dict(EQV2_C4, lmax_list=[6], mmax_list=[2])
    torch.manual_seed(0)
    model = EquiformerV2_nbody(**cfg).to(device).eval()
    loc, vel, mass = initial_states(B, N, rank * B)
    t = lambda x: torch.tensor(x, dtype=torch.float32, device=device)
    loc_d, vel_d, mass_d = t(loc), t(vel), t(mass)
    model.rollout(loc_d, vel_d, mass_d, max(a.warmup, 1) + 1, seed=1)

    def work():
        tp, tv = model.rollout(loc_d, vel_d, mass_d, a.steps + 1, seed=2)
        a.final_states = P.all_gather_shards(torch.cat([tp[:, -1], tv[:, -1]], -1).contiguous())
        return tp
    tp, elapsed = timed_region(work, device, P)
    value = a.steps / elapsed * world
    # roofline: every GEMM launch of one composed forward (a 2-frame rollout after the timed region),
    # event-timed on the launch stream, as the training lines do
    import nbody_amd.segnn_train as ST
    ST.gemm_timer = []
    model.rollout(loc_d, vel_d, mass_d, 2, seed=3)
    torch.cuda.synchronize(device)
    g_ms = sum(e0.elapsed_time(e1) for e0, e1, _ in ST.gemm_timer)
    g_fl, n_g = sum(f for _, _, f in ST.gemm_timer), len(ST.gemm_timer)
    ST.gemm_timer = None
    ach = g_fl / (g_ms * 1e-3) / 1e12 if g_ms > 0 else None
    roof = {"bound": "mfma", "kernel": "gemm_f32 / gemm_f32_batched / grouped (nbx_gemm_f32 family: every SO3_LinearV2, "
                                       "SO(2) convolution and radial linear of the composed forward, each launch timed whole)",
            "achieved": round(ach, 3) if ach else None, "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4) if ach else None, "traffic": None,
            "avg_launch_us": round(1e3 * g_ms / max(n_g, 1), 3), "launches_per_forward": n_g,
            "gflop_per_forward": round(g_fl / 1e9, 4),
            "gemm_share_of_step": round(g_ms * 1e-3 / (elapsed / a.steps), 4),
            "mfma_path": "fp32 MFMA (NBX_GEMM_X3=0)" if os.environ.get("NBX_GEMM_X3", "1")[:1] == "0" else
                         "bf16x3 split MFMA (six bf16 products per fp32 product, fp32 accumulate) for the SO(2) "
                         "convolutions' grouped GEMMs (gemm_x3_ok: >= 2^30 multiply-adds, K >= 64, N >= 96), fp32 "
                         "MFMA for the rest; achieved counts fp32-equivalent flops",
            "timing": "torch.cuda.Event pairs around every GEMM launch of one forward, launch stream"}
    result = {
        "metric": "self-feed rollout steps/sec, EquiformerV2 lmax 6 / mmax 2 N=20 batch=64", "value": round(value, 3),
        "unit": "steps/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(1e3 * elapsed / a.steps, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (GravitySim frame-0 initial states N=20, seeded random-init weights, device-hash edge gauges)",
        "config": {"workload": "EquiformerV2 at the reference default degrees lmax [6] / mmax [2], C4 widths "
                               "(4 layers, sphere 64, attn hidden 64, 4 heads, ffn 64, edge 64), N=20, batch 64 per GPU, "
                               "composed native operators",
                   "model": "EquiformerV2", "global_batch": B * world, "seq_len": a.steps, "parallelism": f"dp{world}"},
        "trajectory_steps_per_s": round(value * B, 1), "roofline": roof,
        "finite": bool(torch.isfinite(tp).all().item())}
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline_eqv2(model, B, B_s=8, cfg=cfg)
    return result


def cpu_baseline_eqv2(model, B_glob, B_s=128, cfg=EQV2_C4):
    from oracle import equiformer_v2 as EQ
    p = {k: v.detach().double().cpu() for k, v in model.named_parameters()}
    loc, vel, mass = initial_states(B_s, 20, 0)
    g = np.random.default_rng(0).uniform(0, 1, (B_s * 20 * 19, 3))
    threads = torch.get_num_threads()
    t0 = time.perf_counter()
    EQ.forward(cfg, p, loc, vel, mass, B_s, 20, g)
    dt = time.perf_counter() - t0
    return {"value": 1.0 / (dt * B_glob / B_s), "unit": "steps/s", "cores": threads, "kind": "port",
            "sample": f"1 forward of B={B_s} systems with the torch fp64 CPU oracle (oracle/equiformer_v2.py), "
                      f"{dt:.2f} s, scaled x{B_glob // B_s} to the B={B_glob} batch; torch threads={threads}"}


# ---------------------------------------------------------------- C5 integrator
def bench_gravity(a, rank, world, device, P):
    from nbody_amd.gravity import GravitySim
    S_glob, N, freq = a.batch or 10000, 100, 10
    T = max(freq, a.steps - a.steps % freq)
    start, S = P.shard_range(S_glob, rank, world)
    sim = GravitySim(n_balls=N, interaction_strength=2, dt=0.01, softening=0.2, device=device)
    # the global batch's initial conditions from one seed, sliced per rank: system i is the same
    # system whatever the rank count (the all-gathered final states equal a one-rank run's)
    rng = np.random.default_rng(0)
    pos = (rng.standard_normal((S_glob, N, 3)) * np.cbrt(N / 5))[start:start + S]
    vel = rng.standard_normal((S_glob, N, 3))[start:start + S]
    vel -= vel.mean(1, keepdims=True)
    mass = np.ones((S, N, 1))
    sim.sample_trajectories(pos, vel, mass, max(freq, a.warmup - a.warmup % freq), freq)

    def work():
        ps, vs, fs = sim.sample_trajectories(pos, vel, mass, T, freq)
        a.final_states = P.all_gather_shards(torch.cat([ps[:, -1], vs[:, -1]], -1).contiguous(), S_glob)
        return ps
    ps, elapsed = timed_region(work, device, P)
    inter = float(S_glob) * N * N * T
    flops = 23.0 * inter        # per pair: 3 sub, 3 fma (r2), +eps, sqrt, mul, div, 3 fma (acc) ~ 23 FP64 ops
    ach = flops / elapsed / world / 1e12
    result = {
        "metric": "ground-truth integrator steps/sec, 10000 systems x N=100", "value": round(T / elapsed, 3),
        "unit": "steps/s", "n_gpus": world, "steps": T, "warmup": a.warmup,
        "ms_per_step": round(1e3 * elapsed / T, 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic (GravitySim-style initial conditions)",
        "config": {"workload": f"C5: GravitySim KDK, {S_glob} systems x N={N}, dt=0.01, G=2, softening=0.2, "
                               f"sample_freq={freq}", "model": "GravitySim", "global_batch": S_glob, "seq_len": T,
                   "parallelism": f"dp{world}"},
        "pair_interactions_per_s": round(inter / elapsed, 1),
        "roofline": {"bound": "valu_f64", "achieved": round(ach, 3), "peak": FP64_VALU_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(ach / FP64_VALU_PEAK_TFLOPS, 4), "traffic": None,
                     "flops_per_pair": 23},
        "finite": bool(torch.isfinite(ps).all().item())}
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline_gravity(T, freq, S_glob)
    return result


def cpu_baseline_gravity(T, freq, S_glob, S_s=4, T_s=2000):
    import ctypes
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "liboracle_gravity.so"))
    N = 100
    rng = np.random.default_rng(0)
    pos = rng.standard_normal((S_s, N, 3))
    vel = rng.standard_normal((S_s, N, 3))
    mass = np.ones((S_s, N))
    outs = [np.zeros((S_s, T_s // freq, N, 3)) for _ in range(3)]
    Pp = lambda x: x.ctypes.data_as(ctypes.c_void_p)
    t0 = time.perf_counter()
    lib.oracle_gravity_sample(ctypes.c_int64(S_s), ctypes.c_int64(N), ctypes.c_int64(T_s), ctypes.c_int64(freq),
                              ctypes.c_double(0.01), ctypes.c_double(2.0), ctypes.c_double(0.2), Pp(pos), Pp(vel),
                              Pp(mass), *[Pp(o) for o in outs])
    dt = time.perf_counter() - t0
    return {"value": T_s / (dt * S_glob / S_s), "unit": "steps/s", "cores": 1, "kind": "port",
            "sample": f"{S_s} systems x {T_s} steps with the C oracle (oracle/gravity.c, 1 core), {dt:.2f} s, "
                      f"scaled to {S_glob} systems"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--model", default="segnn",
                    choices=["segnn", "ponita", "egnn_mc", "egnn_mc_train", "segnn_train", "ponita_train", "eqv2",
                             "eqv2_train", "eqv2_l6", "gravity"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=1)
    ap.add_argument("--cpu-torch-steps", type=int, default=20,
                    help="C2: self-feed steps of the torch CPU restatement timed for cpu_baseline")
    ap.add_argument("--eager", action="store_true",
                    help="egnn_mc_train / segnn_train: run the step eagerly (no HIP graph)")
    ap.add_argument("--deterministic-bn", action="store_true",
                    help="segnn: fixed-order BatchNorm sums (bit-reproducible) instead of fp64 atomics")
    ap.add_argument("--bn-mode", default="batch", choices=["batch", "sync", "running"],
                    help="SEGNN BatchNorm statistics: per-rank batch (default), all-rank SyncBN, running")
    a = ap.parse_args()
    defaults = {"segnn": (200, 20), "ponita": (20, 2), "egnn_mc": (100, 10), "egnn_mc_train": (50, 5),
                "segnn_train": (50, 5), "ponita_train": (30, 3), "eqv2": (20, 2),
                "eqv2_train": (30, 3), "eqv2_l6": (5, 1),
                "gravity": (1000, 100)}
    a.steps = a.steps if a.steps is not None else defaults[a.model][0]
    a.warmup = a.warmup if a.warmup is not None else defaults[a.model][1]

    from nbody_amd import parallel as P
    rank, world, device = P.init_from_env()
    fn = {"segnn": bench_segnn, "ponita": bench_ponita, "egnn_mc": bench_egnn, "egnn_mc_train": bench_egnn_train,
          "segnn_train": bench_segnn_train, "ponita_train": bench_ponita_train, "eqv2_train": bench_eqv2_train,
          "eqv2": bench_eqv2, "eqv2_l6": bench_eqv2_l6, "gravity": bench_gravity}[a.model]
    result = fn(a, rank, world, device, P)
    if rank == 0:
        print(json.dumps(result), flush=True)
    P.barrier()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
