"""CPU checks of the package's general-degree SO(3) constants (so3.py) for lmax <= 6 against the
reference's own construction (tests/golden/eqv2_l6.npz, made by running the reference's SO3_Grid and
SO3_Rotation code: make_eqv2_l6.py) and the oracle's bookkeeping.  The device kernels that consume
them are checked on the GPU (tests/test_gpu_eqv2_general.py)."""
import os

import numpy as np
import pytest
import torch

import nbody_amd._lib as L
from nbody_amd import so3
from nbody_amd.equiformer_v2 import EquiformerV2_nbody
from oracle import e3nn_so3 as E3
from oracle import equiformer_v2 as EQ

HERE = os.path.dirname(os.path.abspath(__file__))
Z6 = np.load(os.path.join(HERE, "golden", "eqv2_l6.npz"))


@pytest.mark.parametrize("lmax,mmax", [(l, m) for l in range(7) for m in range(l + 1)])
def test_layout_matches_coefficient_mapping(lmax, mmax):
    lay, ref = so3.Layout(lmax, mmax), EQ.Layout(lmax, mmax)
    assert lay.sel == ref.sel and lay.red == ref.red and lay.perm == ref.perm and lay.m_size == ref.m_size
    assert [lay.perm[i] for i in lay.inv_perm] == list(range(lay.n_red))
    assert lay.m0 == [i for i, (l, m) in enumerate(lay.red) if m == 0]
    for l in range(lmax + 1):     # get_rotate_inv_rescale (float32-rounded) on the kept columns
        cols = [j for j, (ll, _) in enumerate(lay.red) if ll == l]
        assert (ref.rescale[l * l:(l + 1) ** 2][:, cols] == lay.rescale[l]).all()
    assert lay.dsel_floats == sum(len([1 for (ll, _) in lay.red if ll == l]) * (2 * l + 1) for l in range(lmax + 1))


def test_harmonics_match_oracle():
    u = torch.randn(200, 3, dtype=torch.float64)
    u = u / u.norm(dim=-1, keepdim=True)
    for l in range(7):
        got = torch.stack(so3.sh_component(l, u[:, 0], u[:, 1], u[:, 2]), -1)
        torch.testing.assert_close(got, E3.sh_component(l, u), rtol=0, atol=1e-13)


@pytest.mark.parametrize("lmax", range(7))
def test_grids_match_reference_construction(lmax):
    """SO3_Grid(l, m).to_grid_mat / from_grid_mat for every l <= 6, m <= l, as the reference built them
    (e3nn in float32): agreement to float32 rounding."""
    for m in range(lmax + 1):
        to, fr = so3.so3_grid(lmax, m)
        for got, key in ((to, "to"), (fr, "from")):
            ref = Z6[f"grid/{lmax}{m}/{key}"]
            assert got.shape == ref.shape
            assert np.abs(got.numpy() - ref).max() <= 3e-7 * np.abs(ref).max(), (lmax, m, key)


def test_wigner_table_reproduces_reference_wigner():
    """The device algorithm of nbx_eqv2_wigner restated in numpy on the float32 table: D^l(R) =
    [Y^l(R u_k)]_k P_l equals the reference's Jd-based Wigner blocks (16 frames, l <= 6)."""
    R = Z6["wigner6/rot"]
    D = Z6["wigner6/D"]
    tab = so3.wigner_table(6).double().numpy()
    n = L.c_i64()
    L.check(L.lib().nbx_eqv2_wigner_table_floats(6, n), "nbx_eqv2_wigner_table_floats")
    assert n.value == tab.size == so3.wigner_table_floats(6)
    np.testing.assert_allclose(R[:, :, :], D[:, 1:4, 1:4], atol=1e-12)      # D^1 = R
    off = 0
    for l in range(2, 7):
        K = (l + 1) * (2 * l + 1)
        u = tab[off:off + 3 * K].reshape(K, 3)
        P = tab[off + 3 * K:off + K * (2 * l + 4)].reshape(K, 2 * l + 1)
        off += K * (2 * l + 4)
        v = np.einsum("eab,kb->eka", R, u)
        Y = np.stack(so3.sh_component(l, v[..., 0], v[..., 1], v[..., 2]), -2)
        err = np.abs(Y @ P - D[:, l * l:(l + 1) ** 2, l * l:(l + 1) ** 2]).max()
        assert err <= 1e-6, (l, err)
        assert np.linalg.cond(np.stack(so3.sh_component(l, u[:, 0], u[:, 1], u[:, 2]), 0)) < 2.0
    for lmax in range(7):
        d = L.c_i64()
        for mmax in range(lmax + 1):
            L.check(L.lib().nbx_eqv2_dsel_floats(lmax, mmax, d), "nbx_eqv2_dsel_floats")
            assert d.value == so3.Layout(lmax, mmax).dsel_floats


def test_reference_default_degrees_construct_on_the_composed_path():
    """The constructor default (lmax_list [6], mmax_list [2]) builds; the fused kernels decline it
    and the composed general-degree path takes it.  Multi-resolution lists fail loudly."""
    torch.manual_seed(0)
    m = EquiformerV2_nbody(num_layers=1, sphere_channels=32, attn_hidden_channels=32, ffn_hidden_channels=32,
                           edge_channels=32, num_heads=2, attn_alpha_channels=8, attn_value_channels=4,
                           num_distance_basis=64)
    assert m.lmax_list == [6] and m.mmax_list == [2]
    assert m._native_reason and m._general_reason is None and m.uses_general_ops()
    assert m.blocks[0].norm_1.affine_weight.shape == (7, 32)
    with pytest.raises(NotImplementedError):
        EquiformerV2_nbody(num_layers=1, sphere_channels=32, lmax_list=[4, 2], mmax_list=[2, 2])
