"""Generate the long-horizon C2 SEGNN rollout fixture from the CPU oracle (build container).

    python tests/golden/make_segnn_c2_long.py [--frames 121] [--scale 0.002] [--slice 64] [--add-perturbed]
                                              [--add-perturbed-traj]

Why a second C2 fixture: with random-init weights the C2 rollout of make_segnn_c2.py turns chaotic
within ~5 steps (bodies flung to |pos| ~ 50, pairs passing within 1e-3 of each other), so north_star's
"rollout MSE <= 1e-5 vs reference" can only be checked over that short horizon there.  This fixture
keeps the C2 model and workload -- SEGNN lmax_h=1, hidden 192, 6 layers, N=5, B=1024, train-mode
BatchNorm over the whole batch, GravitySim frame-0 initial states (seeds 0..1023) -- and scales the
output layer ``pre_pool2`` (both 2x1o outputs: the position increment and the new velocity) by
``--scale``, so every step moves a body by ~1e-3 of the inter-body spacing and the autoregressive
map stays close to the identity.  That the horizon is then predictable is shown inside the fixture
(``--add-perturbed``): the fp64 oracle rollout started from initial states one fp32 ulp away -- another
equally valid fp32 rounding of the same physical state -- stays within MSE 1e-7 of it at every frame
(``pert_mse_loc`` / ``pert_mse_vel`` over the stored slice; measured max 5.9e-9 / 5.9e-10 at frame 120:
the input change is amplified ~1e6 over the horizon, smoothly).  Also stored: the same rollout computed
entirely in fp32 arithmetic (``f32_mse_*`` over all 1024 systems), whose position MSE reaches 5.4e-7 by
frame 120 -- numpy's fp32 means over the 20 480 message rows accumulate sequentially (~1e-4 relative),
so it measures that implementation's rounding, not the dynamics.

Generation: ``--frames 121 --scale 0.002`` (31 min fp64 + 58 min fp32 on 8 cores), then
``--add-perturbed`` (43 min).

Stored: the fp32-rounded initial states of all 1024 systems (the device rollout needs the whole
batch: train-mode BatchNorm couples the systems), every frame of the fp64 oracle rollout for the
first ``--slice`` systems (fp64), the per-frame one-ulp sensitivity and fp32-oracle MSEs, the scale and a
weight checksum.  The oracle is the e3nn restatement oracle/segnn.py: parity vs e3nn itself is
UNPINNED (e3nn is absent from this image).

Output: tests/golden/segnn_c2_long.npz
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from make_segnn_c2 import HIDDEN, LAYERS, c2_model, initial_states, weight_checksum  # noqa: E402


def scaled_model(scale):
    model = c2_model()
    with torch.no_grad():
        model.pre_pool2.tp.weight.mul_(scale)
    return model


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=121)
    ap.add_argument("--scale", type=float, default=0.002)
    ap.add_argument("--slice", type=int, default=64)
    ap.add_argument("--add-perturbed", action="store_true",
                    help="add the one-ulp sensitivity (pert_mse_*) to an existing fixture")
    ap.add_argument("--add-perturbed-traj", action="store_true",
                    help="add the one-ulp-perturbed fp64 trajectories of the slice (pert_loc / pert_vel)")
    a = ap.parse_args()
    if a.add_perturbed:
        return add_perturbed()
    if a.add_perturbed_traj:
        return add_perturbed_traj()
    from oracle.rollout import rollout, segnn_step
    from oracle.segnn import SEGNNOracle
    model = scaled_model(a.scale)
    params = {k: t.double().numpy().copy() for k, t in model.state_dict().items()}
    loc, vel, mass = initial_states()
    loc, vel = loc.astype(np.float32).astype(np.float64), vel.astype(np.float32).astype(np.float64)
    om = SEGNNOracle(hidden_features=HIDDEN, num_layers=LAYERS)
    t0 = time.time()
    tl, tv = rollout(segnn_step(om, dict(params), training=True), loc, vel, np.zeros_like(loc), mass, a.frames)
    print(f"fp64 oracle rollout of {a.frames - 1} steps: {time.time() - t0:.1f} s", flush=True)
    p32 = {k: v.astype(np.float32) for k, v in params.items()}
    f32 = lambda x: x.astype(np.float32)
    fl, fv = rollout(segnn_step(om, p32, training=True), f32(loc), f32(vel), f32(np.zeros_like(loc)), f32(mass),
                     a.frames)
    print(f"fp32 oracle rollout done: {time.time() - t0:.1f} s", flush=True)
    mse_l = ((fl.astype(np.float64) - tl) ** 2).mean(axis=(0, 2, 3))
    mse_v = ((fv.astype(np.float64) - tv) ** 2).mean(axis=(0, 2, 3))
    for k in range(0, a.frames, 10):
        print(f"frame {k}: fp32-oracle MSE loc {mse_l[k]:.3e} vel {mse_v[k]:.3e}; mean displacement "
              f"{np.abs(tl[:, k] - tl[:, 0]).mean():.3e}")
    print(f"max fp32-oracle MSE over the horizon: loc {mse_l.max():.3e}, vel {mse_v.max():.3e}")
    S = a.slice
    np.savez_compressed(os.path.join(HERE, "segnn_c2_long.npz"), loc0=loc, vel0=vel,
                        traj_loc=tl[:S], traj_vel=tv[:S], f32_mse_loc=mse_l, f32_mse_vel=mse_v,
                        scale=np.float64(a.scale), weight_checksum=np.float64(weight_checksum(model)))


def add_perturbed():
    """The non-chaos proof that does not depend on how an fp32 computation rounds: the same fp64
    oracle rollout from initial states moved by one fp32 ulp (another equally valid fp32 rounding of
    the same physical state).  Chaotic dynamics amplify that change exponentially; here its MSE over
    the fixture's slice stays at the ulp level (stored per frame as pert_mse_loc / pert_mse_vel).
    (The all-fp32 oracle's position MSE, f32_mse_loc, grows polynomially instead: numpy's fp32 mean
    over the 20 480 message rows of each BatchNorm accumulates sequentially, ~1e-4 relative.)"""
    from oracle.rollout import rollout, segnn_step
    from oracle.segnn import SEGNNOracle
    path = os.path.join(HERE, "segnn_c2_long.npz")
    fx = dict(np.load(path))
    model = scaled_model(float(fx["scale"]))
    assert abs(weight_checksum(model) - float(fx["weight_checksum"])) <= 1e-9 * float(fx["weight_checksum"])
    params = {k: t.double().numpy().copy() for k, t in model.state_dict().items()}
    loc, vel = fx["loc0"], fx["vel0"]
    _, _, mass = initial_states()
    om = SEGNNOracle(hidden_features=HIDDEN, num_layers=LAYERS)
    up = lambda x: np.nextafter(x.astype(np.float32), np.float32(np.inf)).astype(np.float64)
    T = fx["traj_loc"].shape[1]
    t0 = time.time()
    pl, pv = rollout(segnn_step(om, dict(params), training=True), up(loc), up(vel), np.zeros_like(loc), mass, T)
    print(f"perturbed fp64 oracle rollout: {time.time() - t0:.1f} s", flush=True)
    S = fx["traj_loc"].shape[0]
    fx["pert_mse_loc"] = ((pl[:S] - fx["traj_loc"]) ** 2).mean(axis=(0, 2, 3))
    fx["pert_mse_vel"] = ((pv[:S] - fx["traj_vel"]) ** 2).mean(axis=(0, 2, 3))
    for k in range(0, T, 10):
        print(f"frame {k}: one-ulp sensitivity MSE loc {fx['pert_mse_loc'][k]:.3e} vel {fx['pert_mse_vel'][k]:.3e}")
    print(f"max over the horizon: loc {fx['pert_mse_loc'].max():.3e} vel {fx['pert_mse_vel'].max():.3e}")
    np.savez_compressed(path, **fx)


def torch_rollout(params, loc, vel, mass, T):
    """The fp64 train-mode self-feed (infer_self_feed.py:182-194, target pos_dt+vel) on the torch
    restatement oracle/segnn_torch.py (equal to oracle/segnn.py to ~1e-16 per forward, and several
    times faster on the CPU); running statistics carried from step to step."""
    from oracle import segnn_torch as OT
    from oracle.graph import fc_edge_index
    from oracle.segnn import SEGNNOracle
    om = SEGNNOracle(hidden_features=HIDDEN, num_layers=LAYERS)
    P = {k: torch.tensor(v, dtype=torch.float64) for k, v in params.items()}
    Bn, Nn = loc.shape[:2]
    ei = torch.from_numpy(fc_edge_index(Bn, Nn))
    p = torch.tensor(loc.reshape(-1, 3), dtype=torch.float64)
    v = torch.tensor(vel.reshape(-1, 3), dtype=torch.float64)
    m = torch.tensor(mass.reshape(-1, 1), dtype=torch.float64)
    locs, vels = [p.clone()], [v.clone()]
    with torch.no_grad():
        for k in range(T - 1):
            out, stats = OT.forward(om, P, p, v, m, ei, True)
            P.update(stats)
            p, v = p + out[:, :3], out[:, 3:].contiguous()
            locs.append(p.clone())
            vels.append(v.clone())
            if k % 10 == 0:
                print(f"  step {k + 1}/{T - 1}", flush=True)
    st = lambda xs: torch.stack(xs, 1).reshape(Bn, Nn, T, 3).permute(0, 2, 1, 3).numpy()
    return st(locs), st(vels)


def add_perturbed_traj():
    """Store the one-ulp-perturbed fp64 trajectories of the slice (``pert_loc`` / ``pert_vel``), so that
    the device test can normalise any error measure (velocities, displacements pos - pos0, per-system
    relative errors) by the same measure of the reference's own one-ulp sensitivity.  Also re-runs the
    unperturbed rollout on the torch oracle and records its largest difference from the stored numpy
    trajectory (``torch_vs_numpy_max``: the two oracles' ~1e-16 per-step disagreement amplified by the
    horizon), which must stay far below the perturbed rollout's distance."""
    path = os.path.join(HERE, "segnn_c2_long.npz")
    fx = dict(np.load(path))
    model = scaled_model(float(fx["scale"]))
    assert abs(weight_checksum(model) - float(fx["weight_checksum"])) <= 1e-9 * float(fx["weight_checksum"])
    params = {k: t.double().numpy().copy() for k, t in model.state_dict().items()}
    loc, vel = fx["loc0"], fx["vel0"]
    _, _, mass = initial_states()
    T, S = fx["traj_loc"].shape[1], fx["traj_loc"].shape[0]
    up = lambda x: np.nextafter(x.astype(np.float32), np.float32(np.inf)).astype(np.float64)
    t0 = time.time()
    tl, tv = torch_rollout(params, loc, vel, mass, T)
    d = max(np.abs(tl[:S] - fx["traj_loc"]).max(), np.abs(tv[:S] - fx["traj_vel"]).max())
    print(f"torch fp64 rollout: {time.time() - t0:.1f} s; max |torch - numpy| over the slice {d:.3e}", flush=True)
    pl, pv = torch_rollout(params, up(loc), up(vel), mass, T)
    print(f"perturbed torch fp64 rollout: {time.time() - t0:.1f} s", flush=True)
    pm = ((pl[:S] - fx["traj_loc"]) ** 2).mean(axis=(0, 2, 3))
    print(f"pert MSE (torch) vs stored pert_mse_loc: max ratio {np.max(pm[1:] / fx['pert_mse_loc'][1:]):.3f}")
    fx["pert_loc"], fx["pert_vel"] = pl[:S], pv[:S]
    fx["torch_vs_numpy_max"] = np.float64(d)
    np.savez_compressed(path, **fx)


if __name__ == "__main__":
    main()
