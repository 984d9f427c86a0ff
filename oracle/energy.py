"""numpy restatement of Trainer._compute_nbody_energies (trainer.py:888-927) — TEST ORACLE ONLY."""
from __future__ import annotations

import numpy as np


def nbody_energies(loc, vel, G, softening):
    """loc/vel [B, T, N, D] -> dict of batch-mean potential / kinetic / total [T]."""
    loc, vel = np.asarray(loc, dtype=np.float64), np.asarray(vel, dtype=np.float64)
    B, T, n, _ = loc.shape
    kinetic = np.zeros((B, T))
    potential = np.zeros((B, T))
    iu = np.triu_indices(n, 1)
    for b in range(B):
        L, V = loc[b], vel[b]
        kinetic[b] = 0.5 * np.sum(V * V, axis=(1, 2))
        d2 = ((L[:, None, :, :] - L[:, :, None, :]) ** 2).sum(-1)
        r = np.sqrt(d2 + softening * softening)
        r[r > 0] = 1.0 / r[r > 0]
        potential[b] = -G * r[:, iu[0], iu[1]].sum(1)
    pot, kin = potential.mean(0), kinetic.mean(0)
    return {"potential": pot, "kinetic": kin, "total": pot + kin}
