"""Generate the C2-size SEGNN rollout fixture from the CPU oracle (build container).

    python tests/golden/make_segnn_c2.py [--frames 11]

C2 = SEGNN lmax_h=1, hidden 192, 6 layers, N=5, B=1024 (BASELINE.json configs[1]).
Weights: ``torch.manual_seed(0); SEGNN(hidden_features=192, num_layers=6)`` (CPU
RNG, deterministic for the pinned torch of this image; the fixture stores a
checksum the test re-verifies).  Initial states: frame 0 of
``GravitySim(n_balls=5, interaction_strength=2, dt=0.01, softening=0.2)`` with
seeds 0..1023, the reference's sample_trajectory RNG recipe
(synthetic_sim.py:357-381).  Rollout: oracle/rollout.py (infer_self_feed.py:99-194)
in fp64 with train-mode BatchNorm (the reference rollout never calls eval()),
``--frames`` frames, from the fp32-rounded initial states the device path sees; plus
the same rollout from states moved by one fp32 ulp (the reference's own sensitivity:
with random-init weights and batch-coupled train-mode BatchNorm the rollout turns
chaotic within ~5 steps), and the oracle rollout computed entirely in fp32 arithmetic (the
scale of error fp32 rounding alone produces).  The oracle's SEGNN is the e3nn restatement of
oracle/segnn.py: parity vs e3nn itself is UNPINNED (e3nn is absent).

Output: tests/golden/segnn_c2_rollout.npz (trajectories stored as fp32).
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

B, N, HIDDEN, LAYERS = 1024, 5, 192, 6


def c2_model():
    import nbody_amd.segnn as S
    torch.manual_seed(0)
    return S.SEGNN(hidden_features=HIDDEN, num_layers=LAYERS)


def weight_checksum(model):
    return float(sum(t.double().abs().sum().item() for k, t in model.state_dict().items()))


def initial_states():
    from oracle.gravity import initial_conditions
    loc = np.empty((B, N, 3))
    vel = np.empty((B, N, 3))
    for b in range(B):
        loc[b], vel[b], _ = initial_conditions(N, b)
    return loc, vel, np.ones((B, N, 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=11)
    a = ap.parse_args()
    from oracle.rollout import rollout, segnn_step
    from oracle.segnn import SEGNNOracle
    model = c2_model()
    params = {k: t.double().numpy().copy() for k, t in model.state_dict().items()}
    loc, vel, mass = initial_states()
    # the device path consumes fp32 states: the oracle starts from the same fp32-rounded values
    loc, vel = loc.astype(np.float32).astype(np.float64), vel.astype(np.float32).astype(np.float64)
    om = SEGNNOracle(hidden_features=HIDDEN, num_layers=LAYERS)
    t0 = time.time()
    tl, tv = rollout(segnn_step(om, dict(params), training=True), loc, vel, np.zeros_like(loc), mass, a.frames)
    print(f"oracle rollout of {a.frames - 1} steps: {time.time() - t0:.1f} s")
    # the reference's own sensitivity: the same fp64 rollout from initial states moved by one
    # fp32 ulp (another equally valid fp32 rounding of the same physical state)
    up = lambda x: np.nextafter(x.astype(np.float32), np.float32(np.inf)).astype(np.float64)
    pl, pv = rollout(segnn_step(om, dict(params), training=True), up(loc), up(vel), np.zeros_like(loc), mass,
                     a.frames)
    print(f"perturbed oracle rollout done: {time.time() - t0:.1f} s")
    # and the same oracle computed entirely in fp32 arithmetic: how far fp32 rounding alone
    # takes this rollout from the fp64 one (the scale of any fp32 implementation's error)
    p32 = {k: v.astype(np.float32) for k, v in params.items()}
    f32 = lambda x: x.astype(np.float32)
    fl, fv = rollout(segnn_step(om, p32, training=True), f32(loc), f32(vel), f32(np.zeros_like(loc)), f32(mass),
                     a.frames)
    print(f"fp32 oracle rollout done: {time.time() - t0:.1f} s, dtype {fl.dtype}")
    np.savez_compressed(os.path.join(HERE, "segnn_c2_rollout.npz"), loc0=loc, vel0=vel,
                        traj_loc=tl.astype(np.float32), traj_vel=tv.astype(np.float32),
                        pert_loc=pl.astype(np.float32), pert_vel=pv.astype(np.float32),
                        f32_loc=fl.astype(np.float32), f32_vel=fv.astype(np.float32),
                        weight_checksum=np.float64(weight_checksum(model)))


if __name__ == "__main__":
    main()
