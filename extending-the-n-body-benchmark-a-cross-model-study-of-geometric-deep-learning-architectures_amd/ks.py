"""Self-feed macro statistics — drop-in for utils/ks_utils.py (`_ks_p`,
`_combine_pvalues_fisher`) and the energy-threshold / KS part of
Trainer.self_feed_postprocess_common (trainer.py:668-722).

The data-parallel part, the two-sample KS statistic of each (simulation, self-feed)
series pair, runs in libnbx (``nbx_ks_2samp_stat``: NaN drop, bitonic sort in LDS,
empirical CDFs by binary search, bit-exact with scipy.stats.ks_2samp's D); many pairs
go in one launch (e.g. per-system energy series).  The p-value is a scalar function
of (D, n_a, n_b), restated here from scipy 1.15's ks_2samp (method "auto"): exact for
equal sample sizes <= 10000 (the Horner form of Pr(D_{n,n} >= h/n),
_compute_prob_outside_square); other sizes fall back to scipy's own routine on the
host.  Fisher's combination -2 sum log p ~ chi2(2k) uses the closed form of the chi2
survival function for even degrees of freedom, in log space.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _lib

__all__ = ["ks_2samp_stat", "ks_statistic", "ks_pvalue", "_ks_p", "_combine_pvalues_fisher", "ENERGY_ERROR_THRESHOLDS",
           "energy_steps_within", "macro_pvalues"]

ENERGY_ERROR_THRESHOLDS = [2.5, 5]   # trainer.py:27
MAX_AUTO_N = 10000                   # scipy ks_2samp "auto": exact up to this size


def _device():
    return torch.device("cuda", torch.cuda.current_device())


def ks_2samp_stat(a, b, device=None):
    """Batched KS statistics on the device.  a [P, na], b [P, nb] (or 1-D for one pair),
    any array-like -> (D [P] float64 numpy, counts [P, 2] int64 numpy) over the non-NaN
    values."""
    device = device or _device()
    A = torch.as_tensor(np.asarray(a, dtype=np.float64)).to(device)
    Bt = torch.as_tensor(np.asarray(b, dtype=np.float64)).to(device)
    if A.dim() == 1:
        A, Bt = A[None], Bt[None]
    A, Bt = A.contiguous(), Bt.contiguous()
    P = A.shape[0]
    if Bt.shape[0] != P:
        raise ValueError("a and b need the same number of series")
    d = torch.empty(P, dtype=torch.float64, device=device)
    n = torch.empty(P, 2, dtype=torch.int64, device=device)
    _lib.check(_lib.lib().nbx_ks_2samp_stat(_lib.dev_ptr(A), A.shape[1], A.shape[1], _lib.dev_ptr(Bt), Bt.shape[1],
                                            Bt.shape[1], P, _lib.dev_ptr(d), _lib.dev_ptr(n),
                                            _lib.stream_ptr(device)), "nbx_ks_2samp_stat")
    return d.cpu().numpy(), n.cpu().numpy()


def ks_statistic(d: float, n1: int, n2: int) -> float:
    """The statistic scipy's ks_2samp reports for the raw max-CDF gap ``d``: in its exact mode
    (max(n1, n2) <= 10000) d is re-quantised to the lattice h / lcm(n1, n2),
    h = round(d * lcm) (_attempt_exact_2kssamp)."""
    if max(n1, n2) > MAX_AUTO_N:
        return float(d)
    lcm = (n1 // math.gcd(n1, n2)) * n2
    return int(np.round(d * lcm)) * 1.0 / lcm


def _prob_outside_square(n: int, h: int) -> float:
    """Pr(D_{n,n} >= h/n) = 2 (A0 (1 - A1 (1 - A2 (...)))) with A_k the ratio of h-term
    products (scipy _compute_prob_outside_square)."""
    P = 0.0
    k = int(np.floor(n / h))
    while k >= 0:
        p1 = 1.0
        for j in range(h):
            p1 = (n - k * h - j) * p1 / (n + k * h + j + 1)
        P = p1 * (1.0 - P)
        k -= 1
    return 2 * P


def ks_pvalue(d: float, n1: int, n2: int) -> float:
    """Two-sided p-value of ks_2samp for statistic d and sample sizes n1, n2."""
    if n1 == n2 and n1 <= MAX_AUTO_N:
        h = int(np.round(d * n1))          # lcm(n, n) = n
        if h == 0:
            return 1.0
        with np.errstate(invalid="raise", over="raise"):
            try:
                prob = _prob_outside_square(n1, h)
            except FloatingPointError:
                prob = float("nan")
        if 0 <= prob <= 1:
            return float(np.clip(prob, 0, 1))
    # unequal sizes / failed exact path: scipy's own routine from the same statistic
    from scipy.stats._stats_py import _attempt_exact_2kssamp
    from scipy.stats import distributions
    g = math.gcd(n1, n2)
    ok, dd, prob = (_attempt_exact_2kssamp(n1, n2, g, d, "two-sided") if max(n1, n2) <= MAX_AUTO_N
                    else (False, d, float("nan")))
    if not ok:
        m, n = sorted([float(n1), float(n2)], reverse=True)
        prob = distributions.kstwo.sf(d, np.round(m * n / (m + n)))
    return float(np.clip(prob, 0, 1))


def _ks_p(a, b) -> float:
    """utils/ks_utils.py:7-17: NaN-dropped two-sample KS p-value (NaN when a side is empty)."""
    a = np.asarray(a, dtype=np.float64).ravel()
    b = np.asarray(b, dtype=np.float64).ravel()
    if a.size == 0 or b.size == 0:
        return float("nan")
    d, n = ks_2samp_stat(a, b)
    if not (n[0, 0] > 0 and n[0, 1] > 0):
        return float("nan")
    return ks_pvalue(float(d[0]), int(n[0, 0]), int(n[0, 1]))


def _chi2_logsf_even(x: float, dof: int) -> float:
    """log of the chi2 survival function for even dof = 2k: exp(-x/2) sum_{i<k} (x/2)^i / i!."""
    k = dof // 2
    h = x / 2.0
    if h <= 0.0:
        return 0.0
    terms = [i * math.log(h) - math.lgamma(i + 1) for i in range(k)]
    m = max(terms)
    return -h + m + math.log(sum(math.exp(t - m) for t in terms))


def _combine_pvalues_fisher(p_values) -> float:
    """utils/ks_utils.py:20-28: Fisher's method over the finite positive p-values,
    floored at 1e-300 (NaN if none)."""
    vals = [float(p) for p in p_values if p == p and p > 0.0]
    if not vals:
        return float("nan")
    chi_stat = -2.0 * math.fsum(math.log(p) for p in vals)
    combined = math.exp(_chi2_logsf_even(chi_stat, 2 * len(vals)))
    return float(max(combined, 1e-300))


def energy_steps_within(sim_total, sf_total, thresholds=ENERGY_ERROR_THRESHOLDS):
    """trainer.py:693-701: for each threshold t, the last step + 1 where
    1/t < |E_sim / (E_sf + 1e-12)| < t (0 if none)."""
    sim_total = np.asarray(sim_total).reshape(-1)
    sf_total = np.asarray(sf_total).reshape(-1)
    m = min(len(sim_total), len(sf_total))
    ratio = np.abs(sim_total[:m] / (sf_total[:m] + 1e-12))
    out = {}
    for t in thresholds:
        mask = np.where((1.0 / t < ratio) & (ratio < t))[0]
        out[t] = int(mask[-1] + 1) if mask.size > 0 else 0
    return out


def macro_pvalues(energies: dict):
    """trainer.py:707-722 for the N-body energies: per-series KS p-values (total, potential,
    kinetic; all three statistics in ONE device launch) and their Fisher combination."""
    keys = ["total", "potential", "kinetic"]
    sim = [np.asarray(energies["simulation"][k], dtype=np.float64).ravel() for k in keys]
    sf = [np.asarray(energies["self_feed"][k], dtype=np.float64).ravel() for k in keys]
    pvals = {}
    if len({len(x) for x in sim}) == 1 and len({len(x) for x in sf}) == 1 and sim[0].size and sf[0].size:
        d, n = ks_2samp_stat(np.stack(sim), np.stack(sf))
        for i, k in enumerate(keys):
            ok = n[i, 0] > 0 and n[i, 1] > 0
            pvals[f"energy_{k}"] = ks_pvalue(float(d[i]), int(n[i, 0]), int(n[i, 1])) if ok else float("nan")
    else:
        for k, a, b in zip(keys, sim, sf):
            pvals[f"energy_{k}"] = _ks_p(a, b)
    return pvals, _combine_pvalues_fisher(list(pvals.values()))
