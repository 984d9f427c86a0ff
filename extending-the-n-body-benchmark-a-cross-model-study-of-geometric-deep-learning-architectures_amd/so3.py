"""Host-side SO(3) bookkeeping for EquiformerV2 (constant buffers, computed once per model).

* ``coefficient_mapping(lmax_list, mmax_list)``: the buffers of CoefficientMappingModule
  (models/equiformer_v2/architecture/so3.py:30-115): degree / order of every kept coefficient and
  the l-major -> m-major permutation matrix ``to_m``.
* ``Layout(lmax, mmax)``: the same bookkeeping as index lists (kept coefficients, m-primary order,
  per-order sizes) for the composed operators (eqv2_train.py).
* ``so3_grid(lmax, mmax)``: SO3_Grid's to_grid_mat / from_grid_mat (so3.py:543-618) — e3nn's
  ToS2Grid / FromS2Grid with "component" normalisation on the (2(lmax+1)) x (2 mmax + 1 or
  2(mmax+1)+1) equiangular grid, rescaled for l > mmax and restricted to |m| <= mmax.  e3nn is not
  installed; the real spherical harmonics (e3nn basis, lmax <= 6), the grid and the Driscoll-Healy
  quadrature weights are evaluated here in float64 and contracted in float32 like e3nn's
  default-dtype buffers.
* ``wigner_table(lmax)``: the constants the device Wigner kernel (nbx_eqv2_wigner, csrc/eqv2_general.hip)
  needs for degrees 2..lmax: probe unit vectors u_k on a Gauss-Legendre x uniform-alpha product grid
  and P = pinv([Y^l(u_k)]_k), so that D^l(R) = [Y^l(R u_k)]_k P exactly (Y^l(R u) = D^l(R) Y^l(u),
  the relation the reference's Jd-based wigner_D satisfies: SO3_Rotation.set_wigner, so3.py:485-531).

e3nn's real spherical harmonics, y the polar axis, no Condon-Shortley phase:
Y_lm = sqrt(2l+1) sqrt((l-|m|)!/(l+|m|)!) Q_l^|m|(y) {sqrt2 Re (z + i x)^m, 1, sqrt2 Im (z + i x)^|m|}
for m > 0, m = 0, m < 0, with P_l^m = (1 - y^2)^(m/2) Q_l^m ("component" normalisation, sum_m
Y_lm^2 = 2l+1).  For l <= 2 the explicit polynomials are used.

The rotation matrices themselves are computed per edge on the device (csrc/eqv2.hip).
"""
from __future__ import annotations

import math

import numpy as np
import torch

LMAX = 6


def _lm(lmax):
    return [(l, m) for l in range(lmax + 1) for m in range(-l, l + 1)]


def coefficient_mapping(lmax_list, mmax_list):
    """-> dict of float32 tensors l_harmonic, m_harmonic, m_complex, res_size, to_m, m_size."""
    l_h, m_c, res = [], [], []
    for lmax, mmax in zip(lmax_list, mmax_list):
        n0 = len(l_h)
        for l in range(lmax + 1):
            mm = min(mmax, l)
            for m in range(-mm, mm + 1):
                l_h.append(l)
                m_c.append(m)
        res.append(len(l_h) - n0)
    n = len(l_h)
    to_m = torch.zeros(n, n)
    m_size = torch.zeros(max(mmax_list) + 1)
    row = 0
    lmax_all = max(lmax_list)
    for m in range(max(mmax_list) + 1):
        re = [i for i in range(n) if l_h[i] <= lmax_all and m_c[i] == m]
        im = [i for i in range(n) if l_h[i] <= lmax_all and m_c[i] == -m] if m else []
        for i in re + im:
            to_m[row, i] = 1.0
            row += 1
        m_size[m] = len(re)
    f = lambda v: torch.tensor(v, dtype=torch.float32)
    return {"l_harmonic": f(l_h), "m_harmonic": f([abs(m) for m in m_c]), "m_complex": f(m_c),
            "res_size": f(res), "to_m": to_m, "m_size": m_size}


class Layout:
    """Coefficient bookkeeping of one (lmax, mmax) (CoefficientMappingModule, so3.py:30-185):

    * ``sel``: indices of the kept (|m| <= mmax) coefficients among the (lmax+1)^2 l-primary ones
      (coefficient_idx); ``red`` their (l, m);
    * ``perm``: the m-primary order of SO2_Convolution as positions in ``red`` (m = 0 of every l,
      then for m = 1..mmax the +m then the -m coefficients), ``inv_perm`` its inverse;
    * ``m_size[m]`` = lmax - m + 1 coefficients per order;
    * ``m0``: the positions of the m = 0 coefficients in ``red``;
    * ``rescale[l]``: get_rotate_inv_rescale's sqrt((2l+1)/(2 mmax+1)) for l > mmax (float32-rounded,
      as the reference's default-dtype table), 1 otherwise;
    * ``dsel_floats``: floats of one edge's kept Wigner rows, degree blocks [2 min(l, mmax)+1][2l+1].
    """

    def __init__(self, lmax: int, mmax: int):
        if not (0 <= mmax <= lmax <= LMAX):
            raise ValueError(f"need 0 <= mmax <= lmax <= {LMAX}")
        self.lmax, self.mmax = lmax, mmax
        self.full = _lm(lmax)
        self.sel = [i for i, (l, m) in enumerate(self.full) if abs(m) <= mmax]
        self.red = [self.full[i] for i in self.sel]
        perm = []
        for m in range(mmax + 1):
            perm += [i for i, (l, mm) in enumerate(self.red) if mm == m]
            if m:
                perm += [i for i, (l, mm) in enumerate(self.red) if mm == -m]
        self.perm = perm
        self.inv_perm = [perm.index(i) for i in range(len(perm))]
        self.m_size = [lmax - m + 1 for m in range(mmax + 1)]
        self.m0 = [i for i, (l, m) in enumerate(self.red) if m == 0]
        self.rescale = [1.0 if l <= mmax else float(np.float32(math.sqrt((2 * l + 1) / (2 * mmax + 1))))
                        for l in range(lmax + 1)]
        self.dsel_floats = sum((2 * min(l, mmax) + 1) * (2 * l + 1) for l in range(lmax + 1))

    @property
    def n_full(self):
        return (self.lmax + 1) ** 2

    @property
    def n_red(self):
        return len(self.red)


def _legendre_q(l, m, y):
    """Q_l^m(y), P_l^m = (1 - y^2)^(m/2) Q_l^m, no Condon-Shortley phase: Q_m^m = (2m-1)!!,
    Q_{m+1}^m = (2m+1) y Q_m^m, (l-m) Q_l^m = (2l-1) y Q_{l-1}^m - (l+m-1) Q_{l-2}^m."""
    a = np.full_like(y, float(math.prod(range(2 * m - 1, 0, -2))) if m > 0 else 1.0)
    if l == m:
        return a
    b = (2 * m + 1) * y * a
    for k in range(m + 2, l + 1):
        a, b = b, ((2 * k - 1) * y * b - (k + m - 1) * a) / (k - m)
    return b


def sh_component(l, x, y, z):
    """e3nn real spherical harmonics of degree l at unit vectors (x, y, z) (float64 arrays or tensors),
    "component" normalisation -> list of 2l+1 arrays, m = -l..l."""
    if l == 0:
        return [x * 0 + 1.0]
    if l == 1:
        s = math.sqrt(3.0)
        return [s * x, s * y, s * z]
    if l == 2:
        s3, s5 = math.sqrt(3.0), math.sqrt(5.0)
        return [s5 * s3 * x * z, s5 * s3 * x * y, s5 * (y * y - 0.5 * (x * x + z * z)), s5 * s3 * y * z,
                s5 * 0.5 * s3 * (z * z - x * x)]
    if l > LMAX:
        raise NotImplementedError(f"EquiformerV2 supports lmax <= {LMAX}")
    as_t = isinstance(x, torch.Tensor)
    x, y, z = (t.numpy() if as_t else np.asarray(t, dtype=np.float64) for t in (x, y, z))
    re, im = [np.ones_like(x)], [np.zeros_like(x)]              # (z + i x)^m
    for _ in range(l):
        re.append(re[-1] * z - im[-1] * x)
        im.append(re[-2] * x + im[-1] * z)
    out = []
    for m in range(-l, l + 1):
        am = abs(m)
        n = math.sqrt(2 * l + 1) * math.sqrt(math.factorial(l - am) / math.factorial(l + am))
        ang = math.sqrt(2.0) * (re[am] if m > 0 else im[am]) if m else np.ones_like(x)
        out.append(n * _legendre_q(l, am, y) * ang)
    return [torch.from_numpy(o) for o in out] if as_t else out


def _grid_values(lmax, res_beta, res_alpha):
    """Y_i(beta_b, alpha_a) [b, a, i], integral-normalised e3nn real SH on the e3nn S2 grid."""
    beta = (torch.arange(res_beta, dtype=torch.float64) + 0.5) / res_beta * math.pi
    alpha = torch.arange(res_alpha, dtype=torch.float64) / res_alpha * 2 * math.pi
    b, a = torch.meshgrid(beta, alpha, indexing="ij")
    x, y, z = torch.sin(b) * torch.sin(a), torch.cos(b), torch.sin(b) * torch.cos(a)
    ys = [v for l in range(lmax + 1) for v in sh_component(l, x, y, z)]
    return torch.stack(ys, -1) / math.sqrt(4 * math.pi)


def _dh_weights(bw):
    w = []
    for j in range(2 * bw):
        s = sum(math.sin((2 * j + 1) * (2 * k + 1) * math.pi / (4.0 * bw)) / (2 * k + 1) for k in range(bw))
        w.append((2.0 / bw) * math.sin(math.pi * (2.0 * j + 1.0) / (4.0 * bw)) * s)
    return torch.tensor(w, dtype=torch.float64) / (2.0 * (2 * bw) ** 2)


def grid_shape(lmax: int, mmax: int):
    """(res_beta, res_alpha) of SO3_Grid(lmax, mmax) with the default resolution."""
    return 2 * (lmax + 1), (2 * (mmax + 1) + 1 if lmax == mmax else 2 * mmax + 1)


def so3_grid(lmax: int, mmax: int):
    """-> (to_grid_mat, from_grid_mat) float32 [res_beta, res_alpha, n_coeff(|m| <= mmax)]."""
    res_beta, res_alpha = grid_shape(lmax, mmax)
    Y = _grid_values(lmax, res_beta, res_alpha)                           # [b, a, i]
    ls = torch.tensor([l for l, _ in _lm(lmax)], dtype=torch.float64)
    n_to = math.sqrt(4 * math.pi) / torch.sqrt(2 * ls + 1) / math.sqrt(lmax + 1)
    n_from = math.sqrt(4 * math.pi) * torch.sqrt(2 * ls + 1) * math.sqrt(lmax + 1)
    qw = _dh_weights(res_beta // 2) * res_beta ** 2 / res_alpha
    to = (Y * n_to).float()
    fr = (Y * n_from * qw[:, None, None]).float()
    if lmax != mmax:
        for l in range(mmax + 1, lmax + 1):
            s, f = l * l, math.sqrt((2 * l + 1) / (2 * mmax + 1))
            to[:, :, s:s + 2 * l + 1] = to[:, :, s:s + 2 * l + 1] * f
            fr[:, :, s:s + 2 * l + 1] = fr[:, :, s:s + 2 * l + 1] * f
    keep = [i for i, (l, m) in enumerate(_lm(lmax)) if abs(m) <= mmax]
    return to[:, :, keep].contiguous(), fr[:, :, keep].contiguous()


def wigner_probes(l: int):
    """The (l+1)(2l+1) probe unit vectors of degree l: Gauss-Legendre nodes in cos(beta) times
    2l+1 uniform alphas (a product rule exact for degree 2l, so [Y^l(u_k)]_k is well conditioned)."""
    t, _ = np.polynomial.legendre.leggauss(l + 1)
    alpha = 2 * math.pi * np.arange(2 * l + 1) / (2 * l + 1)
    ct, a = np.meshgrid(t, alpha, indexing="ij")
    st = np.sqrt(1 - ct * ct)
    return np.stack([st * np.sin(a), ct, st * np.cos(a)], -1).reshape(-1, 3)


def wigner_table_floats(lmax: int) -> int:
    return sum((l + 1) * (2 * l + 1) * (3 + 2 * l + 1) for l in range(2, lmax + 1))


def wigner_table(lmax: int) -> torch.Tensor:
    """float32 [wigner_table_floats(lmax)]: for l = 2..lmax, u [K][3] then P [K][2l+1] (module docstring)."""
    parts = []
    for l in range(2, lmax + 1):
        u = wigner_probes(l)
        M = np.stack(sh_component(l, u[:, 0], u[:, 1], u[:, 2]), 0)         # [2l+1, K]
        P = np.linalg.pinv(M)                                                # [K, 2l+1]
        parts += [u.reshape(-1), P.reshape(-1)]
    if not parts:
        return torch.zeros(1, dtype=torch.float32)
    out = torch.from_numpy(np.concatenate(parts)).float()
    assert out.numel() == wigner_table_floats(lmax)
    return out
