"""Self-feed macro statistics (utils/ks_utils.py:7-28, trainer.py:668-722).

Oracle: scipy.stats.ks_2samp (the reference's own call, scipy 1.15 in this image) and
the reference's Fisher combination restated with mpmath at 200 digits exactly as
ks_utils.py:20-28 writes it.  CPU: the host p-value / Fisher / threshold code.  GPU:
the device statistic (bit-exact D) and the end-to-end _ks_p."""
import math

import numpy as np
import pytest
from scipy import stats

import nbody_amd.ks as K


def ref_fisher(p_values):
    """ks_utils.py:20-28 (mpmath log-sum, scipy chi2.sf, floor 1e-300)."""
    from mpmath import log, mp
    vals = [p for p in p_values if p == p and p > 0.0]
    if not vals:
        return float("nan")
    mp.dps = 200
    chi_stat = float(-2 * mp.fsum([log(mp.mpf(p)) for p in vals]))
    return float(max(stats.chi2.sf(chi_stat, 2 * len(vals)), 1e-300))


def scipy_d(a, b):
    return stats.ks_2samp(a, b).statistic


def raw_d(a, b):
    """scipy's statistic before its exact-mode lattice re-quantisation: max |cdf1 - cdf2| over
    the concatenated data with searchsorted(side='right') CDFs (ks_2samp body)."""
    sa, sb = np.sort(a), np.sort(b)
    x = np.concatenate([sa, sb])
    return np.abs(np.searchsorted(sa, x, side="right") / a.size - np.searchsorted(sb, x, side="right") / b.size).max()


def check_d(d, a, b):
    assert d == raw_d(a, b)                                   # bit-exact raw statistic
    assert K.ks_statistic(d, a.size, b.size) == scipy_d(a, b)  # and the reported one


@pytest.mark.parametrize("n", [1, 2, 7, 50, 999, 1000, 4096])
def test_pvalue_matches_scipy_equal_sizes(n):
    rng = np.random.default_rng(n)
    for shift in (0.0, 0.05, 0.3, 2.0):
        a = rng.standard_normal(n)
        b = rng.standard_normal(n) + shift
        r = stats.ks_2samp(a, b)
        got = K.ks_pvalue(float(r.statistic), n, n)
        assert got == pytest.approx(float(r.pvalue), rel=1e-12, abs=1e-300), (n, shift)


@pytest.mark.parametrize("n1,n2", [(10, 13), (200, 150), (1000, 20000)])
def test_pvalue_matches_scipy_unequal_sizes(n1, n2):
    rng = np.random.default_rng(n1 + n2)
    a, b = rng.standard_normal(n1), rng.standard_normal(n2) * 1.1
    r = stats.ks_2samp(a, b)
    assert K.ks_pvalue(float(r.statistic), n1, n2) == pytest.approx(float(r.pvalue), rel=1e-10, abs=1e-300)


def test_fisher_matches_reference_formula():
    rng = np.random.default_rng(0)
    cases = [[0.5], [0.01, 0.2, 0.9], [1e-300, 1e-200, 0.5], list(rng.uniform(0, 1, 7)), [float("nan"), 0.0, 0.3],
             [1e-100] * 5, [float("nan")], [], [1.0, 1.0]]
    for c in cases:
        r, g = ref_fisher(c), K._combine_pvalues_fisher(c)
        if r != r:
            assert g != g
        else:
            assert g == pytest.approx(r, rel=1e-12, abs=0), c


def test_energy_threshold_steps():
    sim = np.array([1.0, 1.0, 1.0, 1.0, 1.0])
    sf = np.array([1.0, 0.9, 0.5, 0.1, 0.3])     # ratios 1, 1.1, 2, 10, 3.3
    got = K.energy_steps_within(sim, sf)
    assert got == {2.5: 3, 5: 5}


# ------------------------------------------------------------------ device
@pytest.mark.gpu
def test_device_statistic_bit_exact(hip_device):
    rng = np.random.default_rng(1)
    pairs = []
    for n1, n2 in [(1000, 1000), (1, 1), (3, 5), (4096, 17), (8192, 8192), (100, 100)]:
        a = rng.standard_normal(n1)
        b = rng.standard_normal(n2) * 1.3 + 0.1
        pairs.append((a, b))
    ties = (np.repeat(np.arange(10.0), 30), np.repeat(np.arange(3.0, 13.0), 30))       # heavy ties
    pairs.append(ties)
    for a, b in pairs:
        d, n = K.ks_2samp_stat(a, b, hip_device)
        check_d(d[0], a, b)
        assert tuple(n[0]) == (a.size, b.size)
    # batched, with NaNs dropped as _ks_p does
    A = rng.standard_normal((64, 1000))
    Bm = rng.standard_normal((64, 1000)) + np.linspace(0, 0.5, 64)[:, None]
    A[3, ::7] = np.nan
    Bm[5, :] = np.nan
    d, n = K.ks_2samp_stat(A, Bm, hip_device)
    for p in range(64):
        a, b = A[p][~np.isnan(A[p])], Bm[p][~np.isnan(Bm[p])]
        if b.size == 0:
            assert math.isnan(d[p]) and n[p, 1] == 0
        else:
            check_d(d[p], a, b)
            assert n[p, 0] == a.size


@pytest.mark.gpu
def test_ks_p_and_macros_match_reference(hip_device):
    rng = np.random.default_rng(2)
    T = 1000
    sim = {k: rng.standard_normal(T).cumsum() for k in ("total", "potential", "kinetic")}
    sf = {k: v + rng.standard_normal(T) * 0.5 for k, v in sim.items()}
    pvals, comb = K.macro_pvalues({"simulation": sim, "self_feed": sf})
    ref = {f"energy_{k}": float(stats.ks_2samp(sim[k], sf[k]).pvalue) for k in sim}
    for k, v in ref.items():
        assert pvals[k] == pytest.approx(v, rel=1e-12, abs=1e-300)
    assert comb == pytest.approx(ref_fisher(list(ref.values())), rel=1e-12)
    a = np.r_[rng.standard_normal(50), np.nan, np.nan]
    b = rng.standard_normal(60) + 0.4
    assert K._ks_p(a, b) == pytest.approx(float(stats.ks_2samp(a[:-2], b).pvalue), rel=1e-10, abs=1e-300)
    assert math.isnan(K._ks_p([], [1.0])) and math.isnan(K._ks_p([np.nan], [1.0]))
