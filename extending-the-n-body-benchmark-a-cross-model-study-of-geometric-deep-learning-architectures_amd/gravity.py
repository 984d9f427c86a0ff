"""Drop-in for datasets/nbody/dataset/synthetic_sim.py::GravitySim with the KDK loop
on the device (csrc/gravity.hip, fp64).

Initial conditions use numpy's legacy global RNG exactly like the reference
(sample_trajectory lines 357-381), so a seeded trajectory starts from the same
bits; the T-step integration then runs in one kernel for all systems at once.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib


class GravitySim:
    def __init__(self, n_balls=100, loc_std=1, vel_norm=0.5, interaction_strength=1, noise_var=0, dt=0.001,
                 softening=0.1, dim=3, device="cuda"):
        self.n_balls, self.loc_std, self.vel_norm = n_balls, loc_std, vel_norm
        self.interaction_strength, self.noise_var, self.dt = interaction_strength, noise_var, dt
        self.softening, self.dim = softening, dim
        self.device = torch.device(device)
        if dim != 3:
            raise NotImplementedError("GravitySim HIP path is 3-D")

    # ---------------------------------------------------------------- physics
    @staticmethod
    def compute_acceleration(pos, mass, G, softening):
        """synthetic_sim.py:318-340 for pos [..., N, 3] (numpy or torch), on the device."""
        as_numpy = isinstance(pos, np.ndarray)
        p = torch.as_tensor(pos, dtype=torch.float64)
        m = torch.as_tensor(mass, dtype=torch.float64)
        dev = p.device if p.is_cuda else torch.device("cuda")
        N = p.shape[-2]
        S = p.numel() // (3 * N)
        pd = p.reshape(S, N, 3).to(dev).contiguous()
        md = m.reshape(S, N).to(dev).contiguous()
        acc = torch.empty_like(pd)
        _lib.check(_lib.lib().nbx_gravity_acceleration(_lib.dev_ptr(pd), _lib.dev_ptr(md), S, N, float(G),
                                                       float(softening), _lib.dev_ptr(acc), _lib.stream_ptr(dev)),
                   "nbx_gravity_acceleration")
        acc = acc.reshape(p.shape)
        return acc.cpu().numpy() if as_numpy else acc

    @staticmethod
    def compute_force(pos, mass, G, softening, batch_size=None):
        """synthetic_sim.py:422-448."""
        if batch_size is None:
            return GravitySim.compute_acceleration(pos, mass, G, softening) * mass
        rows = pos.shape[0]
        if rows % batch_size != 0:
            raise ValueError(f"batch_size {batch_size} is not a divisor of the number of particles {rows}.")
        nb = rows // batch_size
        p = pos.reshape(batch_size, nb, -1)
        m = mass.reshape(batch_size, nb, -1)
        acc = GravitySim.compute_acceleration(p, m, G, softening) * m
        return acc.reshape(-1, 3)

    def initial_conditions(self, random_seed):
        """synthetic_sim.py:357-381 (legacy np.random, per-trajectory seed)."""
        np.random.seed(random_seed)
        N = self.n_balls
        mass = np.ones((N, 1))
        pos = np.random.randn(N, self.dim) * np.cbrt(N / 5)
        vel = np.random.randn(N, self.dim)
        vel -= np.mean(mass * vel, 0) / np.mean(mass)
        return pos, vel, mass

    def sample_trajectories(self, pos, vel, mass, T=10000, sample_freq=10):
        """Batched KDK loop (synthetic_sim.py:383-408) for S systems at once.
        pos/vel [S,N,3], mass [S,N,1] (numpy or torch) -> device tensors
        (pos_save, vel_save, force_save) [S, T/sample_freq, N, 3] fp64."""
        assert T % sample_freq == 0
        dev = self.device
        p = torch.as_tensor(pos, dtype=torch.float64).to(dev).contiguous().clone()
        v = torch.as_tensor(vel, dtype=torch.float64).to(dev).contiguous().clone()
        S, N, _ = p.shape
        m = torch.as_tensor(mass, dtype=torch.float64).reshape(S, N).to(dev).contiguous()
        Ts = T // sample_freq
        ps = torch.empty(S, Ts, N, 3, dtype=torch.float64, device=dev)
        vs, fs = torch.empty_like(ps), torch.empty_like(ps)
        _lib.check(_lib.lib().nbx_gravity_sample(
            _lib.dev_ptr(p), _lib.dev_ptr(v), _lib.dev_ptr(m), S, N, T, sample_freq, float(self.dt),
            float(self.interaction_strength), float(self.softening), _lib.dev_ptr(ps), _lib.dev_ptr(vs),
            _lib.dev_ptr(fs), _lib.stream_ptr(dev)), "nbx_gravity_sample")
        return ps, vs, fs

    def sample_trajectory(self, T=10000, sample_freq=10, og_pos_save=None, og_vel_save=None, og_force_save=None,
                          random_seed=None, log_progress=False):
        """synthetic_sim.py:357-420 for one trajectory; returns numpy arrays like the reference."""
        if og_pos_save is not None:
            raise NotImplementedError("continuation runs (og_*_save) are outside the native path")
        pos, vel, mass = self.initial_conditions(random_seed)
        ps, vs, fs = self.sample_trajectories(pos[None], vel[None], mass[None], T, sample_freq)
        out = [t[0].cpu().numpy() for t in (ps, vs, fs)]
        Ts = T // sample_freq
        for o in out:  # the reference draws the observation noise even when noise_var == 0
            o += np.random.randn(Ts, self.n_balls, self.dim) * self.noise_var
        return out[0], out[1], out[2], mass

    def sample_trajectory_batch(self, batch_size, T=10000, sample_freq=10, seeds=None, shard=False):
        """``batch_size`` independent ``sample_trajectory`` calls integrated in one launch.
        Each trajectory consumes the legacy RNG exactly as the reference's does
        (seed -> initial conditions -> observation noise; the integration itself draws
        nothing), so trajectory i equals ``sample_trajectory(random_seed=seeds[i])``.
        ``seeds=None`` means OS entropy per trajectory, like the reference dataset.

        ``shard=True`` under torch.distributed (one process per GPU; the reference's
        ProcessPool, dataset_gravity_otf.py:96-104, spread over GPUs): each rank integrates
        its contiguous block of the trajectories (parallel.shard_range) and one all-gather
        (RCCL over xGMI) gives every rank the whole batch in trajectory order."""
        from . import parallel as P
        if seeds is None:
            seeds = [None] * batch_size
        if len(seeds) != batch_size:
            raise ValueError("need one seed per trajectory")
        world = P.world() if shard else 1
        start, count = P.shard_range(batch_size, P.rank(), world) if world > 1 else (0, batch_size)
        Ts = T // sample_freq
        ics = []
        for s in seeds[start:start + count]:
            pos, vel, mass = self.initial_conditions(s)
            nz = [np.random.randn(Ts, self.n_balls, self.dim) * self.noise_var for _ in range(3)]
            ics.append((pos, vel, mass, nz))
        N = self.n_balls
        pos = np.stack([c[0] for c in ics]) if ics else np.zeros((0, N, 3))
        vel = np.stack([c[1] for c in ics]) if ics else np.zeros((0, N, 3))
        mass = np.stack([c[2] for c in ics]) if ics else np.zeros((0, N, 1))
        if count:
            ps, vs, fs = self.sample_trajectories(pos, vel, mass, T, sample_freq)
        else:
            ps = vs = fs = torch.zeros(0, Ts, N, 3, dtype=torch.float64, device=self.device)
        if ics and self.noise_var:
            noise = torch.as_tensor(np.stack([np.stack(c[3]) for c in ics]), device=self.device)   # [S, 3, Ts, N, 3]
            ps, vs, fs = ps + noise[:, 0], vs + noise[:, 1], fs + noise[:, 2]
        m = torch.as_tensor(mass, dtype=torch.float64, device=self.device)
        if world > 1:
            ps, vs, fs, m = (P.all_gather_shards(t.contiguous(), batch_size) for t in (ps, vs, fs, m))
        ps, vs, fs, m = (t.cpu().numpy() for t in (ps, vs, fs, m))
        return [(ps[i], vs[i], fs[i], m[i]) for i in range(batch_size)]

    def _energy(self, pos, vel, mass, G):
        """synthetic_sim.py:450-473 (host numpy, evaluation only)."""
        KE = 0.5 * np.sum(np.sum(mass * vel ** 2))
        d = pos[None, :, :] - pos[:, None, :]
        inv_r = np.sqrt((d ** 2).sum(-1) + self.softening ** 2)
        inv_r[inv_r > 0] = 1.0 / inv_r[inv_r > 0]
        PE = G * np.sum(np.triu(-(mass * mass.T) * inv_r, 1))
        return KE, PE, KE + PE
