"""Host-side SO(3) bookkeeping for EquiformerV2 (constant buffers, computed once per model).

* ``coefficient_mapping(lmax_list, mmax_list)``: the buffers of CoefficientMappingModule
  (models/equiformer_v2/architecture/so3.py:30-115): degree / order of every kept coefficient and
  the l-major -> m-major permutation matrix ``to_m``.
* ``so3_grid(lmax, mmax)``: SO3_Grid's to_grid_mat / from_grid_mat (so3.py:543-618) — e3nn's
  ToS2Grid / FromS2Grid with "component" normalisation on the (2(lmax+1)) x (2 mmax + 1 or
  2(mmax+1)+1) equiangular grid, rescaled for l > mmax and restricted to |m| <= mmax.  e3nn is not
  installed; the real spherical harmonics (e3nn basis, lmax <= 2), the grid and the Driscoll-Healy
  quadrature weights are evaluated here in float64 and contracted in float32 like e3nn's
  default-dtype buffers.

The rotation matrices themselves are computed per edge on the device (csrc/eqv2.hip).
"""
from __future__ import annotations

import math

import torch

LMAX = 2


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


def _sh_component(l, x, y, z):
    if l == 0:
        return [torch.ones_like(x)]
    if l == 1:
        s = math.sqrt(3.0)
        return [s * x, s * y, s * z]
    if l == 2:
        s3, s5 = math.sqrt(3.0), math.sqrt(5.0)
        return [s5 * s3 * x * z, s5 * s3 * x * y, s5 * (y * y - 0.5 * (x * x + z * z)), s5 * s3 * y * z,
                s5 * 0.5 * s3 * (z * z - x * x)]
    raise NotImplementedError(f"EquiformerV2 native path supports lmax <= {LMAX}")


def _grid_values(lmax, res_beta, res_alpha):
    """Y_i(beta_b, alpha_a) [b, a, i], integral-normalised e3nn real SH on the e3nn S2 grid."""
    beta = (torch.arange(res_beta, dtype=torch.float64) + 0.5) / res_beta * math.pi
    alpha = torch.arange(res_alpha, dtype=torch.float64) / res_alpha * 2 * math.pi
    b, a = torch.meshgrid(beta, alpha, indexing="ij")
    x, y, z = torch.sin(b) * torch.sin(a), torch.cos(b), torch.sin(b) * torch.cos(a)
    ys = [v for l in range(lmax + 1) for v in _sh_component(l, x, y, z)]
    return torch.stack(ys, -1) / math.sqrt(4 * math.pi)


def _dh_weights(bw):
    w = []
    for j in range(2 * bw):
        s = sum(math.sin((2 * j + 1) * (2 * k + 1) * math.pi / (4.0 * bw)) / (2 * k + 1) for k in range(bw))
        w.append((2.0 / bw) * math.sin(math.pi * (2.0 * j + 1.0) / (4.0 * bw)) * s)
    return torch.tensor(w, dtype=torch.float64) / (2.0 * (2 * bw) ** 2)


def so3_grid(lmax: int, mmax: int):
    """-> (to_grid_mat, from_grid_mat) float32 [res_beta, res_alpha, n_coeff(|m| <= mmax)]."""
    res_beta = 2 * (lmax + 1)
    res_alpha = 2 * (mmax + 1) + 1 if lmax == mmax else 2 * mmax + 1
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
