"""numpy restatement of GravitySim (datasets/nbody/dataset/synthetic_sim.py:305-473)
— TEST ORACLE ONLY.  Vectorised over a leading systems axis; per system the
arithmetic follows the reference expression by expression."""
from __future__ import annotations

import numpy as np


def initial_conditions(n_balls: int, random_seed, dim: int = 3):
    """sample_trajectory lines 357-381: legacy np.random global RNG, seeded per
    trajectory; pos ~ randn * cbrt(N/5); vel ~ randn minus the CoM velocity;
    mass = 1.  Returns (pos[N,3], vel[N,3], mass[N,1]) in fp64."""
    np.random.seed(random_seed)
    mass = np.ones((n_balls, 1))
    std_dev = np.cbrt(n_balls / 5)
    pos = np.random.randn(n_balls, dim) * std_dev
    vel = np.random.randn(n_balls, dim)
    vel -= np.mean(mass * vel, 0) / np.mean(mass)
    return pos, vel, mass


def compute_acceleration(pos, mass, G, softening):
    """compute_acceleration (318-340) for pos [..., N, 3], mass [..., N, 1]."""
    x, y, z = pos[..., 0:1], pos[..., 1:2], pos[..., 2:3]
    dx = np.swapaxes(x, -1, -2) - x
    dy = np.swapaxes(y, -1, -2) - y
    dz = np.swapaxes(z, -1, -2) - z
    inv_r3 = dx ** 2 + dy ** 2 + dz ** 2 + softening ** 2
    pos_mask = inv_r3 > 0
    inv_r3[pos_mask] = inv_r3[pos_mask] ** (-1.5)
    ax = G * (dx * inv_r3) @ mass
    ay = G * (dy * inv_r3) @ mass
    az = G * (dz * inv_r3) @ mass
    return np.concatenate((ax, ay, az), axis=-1)


def simulate_step(pos, vel, acc, mass, dt, G, softening):
    """simulate_step (342-355): kick / drift / recompute / kick."""
    vel = vel + acc * dt / 2.0
    pos = pos + vel * dt
    acc = compute_acceleration(pos, mass, G, softening)
    vel = vel + acc * dt / 2.0
    return pos, vel, acc


def sample_trajectories(pos, vel, mass, T=10000, sample_freq=10, dt=0.01, G=2.0, softening=0.2):
    """sample_trajectory loop (383-408) from given initial states (noise_var=0).
    pos/vel [S, N, 3], mass [S, N, 1] -> (pos_save, vel_save, force_save)
    each [S, T/sample_freq, N, 3]."""
    assert T % sample_freq == 0
    S, N, D = pos.shape
    T_save = T // sample_freq
    pos_save = np.zeros((S, T_save, N, D))
    vel_save = np.zeros((S, T_save, N, D))
    force_save = np.zeros((S, T_save, N, D))
    pos, vel = pos.copy(), vel.copy()
    acc = compute_acceleration(pos, mass, G, softening)
    c = 0
    for i in range(T):
        if i % sample_freq == 0:
            pos_save[:, c] = pos
            vel_save[:, c] = vel
            force_save[:, c] = acc * mass
            c += 1
        pos, vel, acc = simulate_step(pos, vel, acc, mass, dt, G, softening)
    return pos_save, vel_save, force_save


def energy(pos, vel, mass, G, softening):
    """GravitySim._energy (450-473) for one frame [N,3]: (KE, PE, total)."""
    KE = 0.5 * np.sum(np.sum(mass * vel ** 2))
    x, y, z = pos[:, 0:1], pos[:, 1:2], pos[:, 2:3]
    dx, dy, dz = x.T - x, y.T - y, z.T - z
    inv_r = np.sqrt(dx ** 2 + dy ** 2 + dz ** 2 + softening ** 2)
    inv_r[inv_r > 0] = 1.0 / inv_r[inv_r > 0]
    PE = G * np.sum(np.sum(np.triu(-(mass * mass.T) * inv_r, 1)))
    return KE, PE, KE + PE
