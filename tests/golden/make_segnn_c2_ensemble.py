"""Generate the C2 rollout *ensemble* fixture: many equally valid fp32 computations of the same
10-step C2 rollout (build container, CPU only).

    python tests/golden/make_segnn_c2_ensemble.py [--procs 8]

Why: the C2 rollout of tests/golden/make_segnn_c2.py turns chaotic after ~5 steps (random-init
weights; system 595 passes a near-collision at step 6 and train-mode BatchNorm couples every
system to it), so past that horizon one fp32 oracle sample cannot say whether a device path is
"another valid rounding" or "systematically worse".  This script computes an ensemble of fp32
rollouts that differ only in rounding -- each one a correct fp32 evaluation of the reference
algorithm (helper_scripts/infer_self_feed.py:99-194 over models/segnn/segnn.py:150-304) -- and stores,
per member and step, the MSE against the fp64 oracle rollout of segnn_c2_rollout.npz and the
per-system error profile.  tests/test_gpu_segnn.py::test_rollout_c2_matches_oracle_fixture then
requires the device rollout to sit inside the ensemble at every step past the horizon.

Members (all from the same fp32-rounded initial states unless stated):
  * ``numpy-fp32``      the numpy oracle in fp32 arithmetic (segnn_c2_rollout.npz ``f32_*``);
  * ``torch-fp32``      the torch restatement oracle/segnn_torch.py in fp32 (cascade reductions,
                        einsum + matmul GEMMs: other summation orders than numpy's);
  * ``sysperm-i``       torch fp32 on the batch with its systems permuted (the BatchNorm sums and
                        the GEMM row blocking run in another order), outputs permuted back;
  * ``edgeperm-i``      torch fp32 on the fully connected edge list in a shuffled order (the
                        aggregation at each destination sums its 4 messages in another order);
  * ``kperm-i``         torch fp32 with the contraction axis of every tensor-product GEMM permuted
                        (the same products summed in another order);
  * ``ulp-i``           torch fp32 from initial states where a random quarter of the systems is
                        rounded to the neighbouring fp32 value (another valid fp32 rounding of the
                        same GravitySim state);
  * ``fp64-ulp-i``      torch fp64 from such states (the reference's own sensitivity);
  * ``fp64-ulp-all``    the numpy fp64 oracle from states all one ulp up (segnn_c2_rollout.npz ``pert_*``).

Stored per member m, step k: ``mse_loc[m, k]``, ``mse_vel[m, k]`` and ``sys_err[m, k, s]`` (max over
system s's bodies / components of |x - fp64| divided by max |fp64| of the frame, positions), plus the
member names.  The oracle is the e3nn restatement: parity vs e3nn itself is UNPINNED (e3nn absent).

Output: tests/golden/segnn_c2_ensemble.npz
"""
from __future__ import annotations

import argparse
import multiprocessing as mp
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from make_segnn_c2 import HIDDEN, LAYERS, B, N, c2_model  # noqa: E402


def _fctp_kperm(rng):
    """oracle/segnn_torch.fctp with the (u, v) contraction axis of each instruction permuted."""
    from oracle.e3nn_lite import wigner_3j

    def fctp(tp, x1, x2, w):
        Z = x1.shape[0]
        s1, s2, so = tp.irreps_in1.slices(), tp.irreps_in2.slices(), tp.irreps_out.slices()
        parts = [[] for _ in tp.irreps_out]
        off = 0
        for (i1, i2, io, (m1, m2, mo)), c in zip(tp.instructions, tp.coeffs):
            n = m1 * m2 * mo
            W = w[off:off + n].reshape(m1 * m2, mo)
            off += n
            d1, d2, do = tp.irreps_in1[i1][1].dim, tp.irreps_in2[i2][1].dim, tp.irreps_out[io][1].dim
            C = torch.as_tensor(wigner_3j(tp.irreps_in1[i1][1].l, tp.irreps_in2[i2][1].l, tp.irreps_out[io][1].l),
                                dtype=x1.dtype)
            a = x1[:, s1[i1]].reshape(Z, m1, d1)
            b = x2[:, s2[i2]].reshape(Z, m2, d2)
            t = torch.einsum("zui,zvj,ijk->zkuv", a, b, C).reshape(Z, do, m1 * m2)
            perm = torch.as_tensor(rng.permutation(m1 * m2))
            y = (t[:, :, perm] @ W[perm]).permute(0, 2, 1).reshape(Z, mo * do)
            parts[io].append(c * y)
        out = [sum(p) if p else x1.new_zeros(Z, so[io].stop - so[io].start) for io, p in enumerate(parts)]
        return torch.cat(out, 1)
    return fctp


def member_rollout(spec):
    """One ensemble member: (name, loc [B, T, N, 3] fp64, vel)."""
    name, kind, seed, dtype_s, frames = spec
    torch.set_num_threads(1)
    import oracle.segnn_torch as ST
    from oracle.graph import fc_edge_index
    from oracle.segnn import SEGNNOracle
    fx = np.load(os.path.join(HERE, "segnn_c2_rollout.npz"))
    dt = torch.float64 if dtype_s == "f64" else torch.float32
    rng = np.random.default_rng(seed)
    model = c2_model()
    P = {k: t.to(dt) for k, t in model.state_dict().items()}
    om = SEGNNOracle(hidden_features=HIDDEN, num_layers=LAYERS)
    loc, vel = fx["loc0"].copy(), fx["vel0"].copy()          # fp32-rounded values held in fp64
    if kind == "ulp":
        sel = rng.random(B) < 0.25
        sgn = np.where(rng.random((B, N, 3)) < 0.5, -np.inf, np.inf).astype(np.float32)
        for arr in (loc, vel):
            moved = np.nextafter(arr.astype(np.float32), sgn).astype(np.float64)
            arr[sel] = moved[sel]
    perm = rng.permutation(B) if kind == "sysperm" else np.arange(B)
    inv = np.argsort(perm)
    ei = fc_edge_index(B, N)
    if kind == "edgeperm":
        ei = ei[:, rng.permutation(ei.shape[1])]
    ei = torch.as_tensor(ei)
    fctp_saved = ST.fctp
    if kind == "kperm":
        ST.fctp = _fctp_kperm(rng)
    try:
        l = torch.tensor(loc[perm].reshape(B * N, 3), dtype=dt)
        v = torch.tensor(vel[perm].reshape(B * N, 3), dtype=dt)
        m = torch.ones(B * N, 1, dtype=dt)
        locs, vels = [l], [v]
        with torch.no_grad():
            for _ in range(frames - 1):
                out, stats = ST.forward(om, P, l, v, m, ei, True)
                P.update(stats)
                l = l + out[:, :3]
                v = out[:, 3:].contiguous()
                locs.append(l)
                vels.append(v)
    finally:
        ST.fctp = fctp_saved
    tl = torch.stack(locs, 0).reshape(frames, B, N, 3).double().numpy()[:, inv].transpose(1, 0, 2, 3)
    tv = torch.stack(vels, 0).reshape(frames, B, N, 3).double().numpy()[:, inv].transpose(1, 0, 2, 3)
    return name, tl, tv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=8)
    a = ap.parse_args()
    fx = np.load(os.path.join(HERE, "segnn_c2_rollout.npz"))
    rl, rv = fx["traj_loc"].astype(np.float64), fx["traj_vel"].astype(np.float64)
    T = rl.shape[1]
    specs = [("torch-fp32", "plain", 0, "f32", T)]
    specs += [(f"sysperm-{i}", "sysperm", 100 + i, "f32", T) for i in range(10)]
    specs += [(f"edgeperm-{i}", "edgeperm", 200 + i, "f32", T) for i in range(8)]
    specs += [(f"kperm-{i}", "kperm", 300 + i, "f32", T) for i in range(8)]
    specs += [(f"ulp-{i}", "ulp", 400 + i, "f32", T) for i in range(8)]
    specs += [(f"fp64-ulp-{i}", "ulp", 500 + i, "f64", T) for i in range(4)]
    t0 = time.time()
    with mp.get_context("spawn").Pool(a.procs) as pool:
        runs = pool.map(member_rollout, specs, chunksize=1)
    print(f"{len(runs)} members in {time.time() - t0:.0f} s")
    runs = [("numpy-fp32", fx["f32_loc"].astype(np.float64), fx["f32_vel"].astype(np.float64))] + runs
    runs += [("fp64-ulp-all", fx["pert_loc"].astype(np.float64), fx["pert_vel"].astype(np.float64))]
    names = [r[0] for r in runs]
    M = len(runs)
    mse_loc, mse_vel = np.zeros((M, T)), np.zeros((M, T))
    sys_err = np.zeros((M, T, B), dtype=np.float32)
    for i, (_, tl, tv) in enumerate(runs):
        for k in range(T):
            mse_loc[i, k] = ((tl[:, k] - rl[:, k]) ** 2).mean()
            mse_vel[i, k] = ((tv[:, k] - rv[:, k]) ** 2).mean()
            sys_err[i, k] = np.abs(tl[:, k] - rl[:, k]).reshape(B, -1).max(1) / np.abs(rl[:, k]).max()
        print(f"{names[i]:>14}: MSE pos per step " + " ".join(f"{x:.1e}" for x in mse_loc[i, 1:]))
    np.savez_compressed(os.path.join(HERE, "segnn_c2_ensemble.npz"), names=np.array(names),
                        mse_loc=mse_loc, mse_vel=mse_vel, sys_err=sys_err,
                        weight_checksum=fx["weight_checksum"])


if __name__ == "__main__":
    main()
