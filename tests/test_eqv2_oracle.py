"""EquiformerV2 oracle vs the reference's own outputs (tests/golden/eqv2.npz, made by
tests/golden/make_eqv2.py running models/equiformer_v2 on test-only e3nn / PyG shims)."""
import json
import os
import sys

import numpy as np
import pytest
import torch

from oracle import e3nn_so3 as E
from oracle import equiformer_v2 as EQ

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from eqv2_params import param_value  # noqa: E402

Z = np.load(os.path.join(HERE, "golden", "eqv2.npz"))
STATE = json.load(open(os.path.join(HERE, "golden", "eqv2_state.json")))


def params(tag):
    """The generator copied param_value into the (float32-built) reference model before .to(dtype)."""
    return {k: torch.from_numpy(param_value(k, STATE[tag]["keys"][k])).float().double() for k in STATE[tag]["params"]}


def test_wigner_matches_reference_jd():
    R = torch.from_numpy(Z["wigner/rot"])
    D = torch.from_numpy(Z["wigner/D"])
    np.testing.assert_allclose(EQ.wigner(R, 2).numpy(), D.numpy(), atol=2e-7)   # the y-pole edge: acos limits the ref


def test_grid_matrices_match_reference_construction():
    for l in range(3):
        for m in range(l + 1):
            to, fr = EQ.grid_mats(l, m)
            np.testing.assert_allclose(to.numpy(), Z[f"grid/{l}{m}/to"], rtol=0, atol=1e-14)
            np.testing.assert_allclose(fr.numpy(), Z[f"grid/{l}{m}/from"], rtol=0, atol=1e-14)


def test_grid_round_trip_exact():
    """The restated e3nn grid (float64 construction) inverts exactly on band-limited signals."""
    for lmax in range(3):
        rb, ra = 2 * (lmax + 1), 2 * (lmax + 1) + 1
        to, fr = E.ToS2Grid(lmax, (rb, ra), dtype=torch.float64), E.FromS2Grid((rb, ra), lmax, dtype=torch.float64)
        tm = torch.einsum("mbi,am->bai", to.shb, to.sha)
        fm = torch.einsum("am,mbi->bai", fr.sha, fr.shb)
        np.testing.assert_allclose(torch.einsum("bai,bak->ik", fm, tm).numpy(), np.eye((lmax + 1) ** 2), atol=1e-13)


@pytest.mark.parametrize("tag", ["c4", "inf"])
def test_forward_matches_reference(tag):
    cfg = STATE[tag]["config"]
    loc, vel, mass = Z[f"{tag}/loc"], Z[f"{tag}/vel"], Z[f"{tag}/mass"]
    B, N = loc.shape[:2]
    acts = {}
    pred = EQ.forward(cfg, params(tag), loc, vel, mass, B, N, Z[f"{tag}/gauge"], acts=acts)
    ref = Z[f"{tag}/f64/pred"]
    np.testing.assert_allclose(pred.numpy(), ref, rtol=1e-9, atol=1e-10)
    for k in ("edge_degree", "block0", "final_norm"):
        np.testing.assert_allclose(acts[k].numpy(), Z[f"{tag}/f64/{k}"], rtol=1e-9, atol=1e-10)


def test_rollout_matches_reference():
    cfg = STATE["c4"]["config"]
    L, V = EQ.rollout(cfg, params("c4"), Z["roll/loc0"], Z["roll/vel0"], Z["roll/mass"], Z["roll/loc"].shape[1],
                      Z["roll/gauge"])
    np.testing.assert_allclose(L.numpy(), Z["roll/loc"], rtol=1e-9, atol=1e-10)
    np.testing.assert_allclose(V.numpy(), Z["roll/vel"], rtol=1e-9, atol=1e-10)


def test_rotation_conventions():
    """D^1 = R and Y(R u) = D(R) Y(u) (the properties the reference's Jd-based Wigner-D satisfies)."""
    g = torch.Generator().manual_seed(0)
    R = EQ.edge_rot_mat(torch.randn(6, 3, dtype=torch.float64, generator=g),
                        torch.rand(6, 3, dtype=torch.float64, generator=g))
    assert torch.allclose(R @ R.transpose(1, 2), torch.eye(3, dtype=torch.float64).expand(6, 3, 3), atol=1e-14)
    assert torch.allclose(torch.linalg.det(R), torch.ones(6, dtype=torch.float64))
    u = torch.nn.functional.normalize(torch.randn(5, 3, dtype=torch.float64, generator=g), dim=-1)
    for l in range(3):
        D = E.wigner_from_matrix(R, l)
        lhs = E.sh_component(l, torch.einsum("nij,kj->nki", R, u))
        rhs = torch.einsum("nij,kj->nki", D, E.sh_component(l, u))
        assert torch.allclose(lhs, rhs, atol=1e-13)


# ---------------------------------------------------------------- lmax > 2 (reference default degrees)
Z6 = np.load(os.path.join(HERE, "golden", "eqv2_l6.npz"))
STATE6 = json.load(open(os.path.join(HERE, "golden", "eqv2_l6_state.json")))


def params6(tag):
    return {k: torch.from_numpy(param_value(k, STATE6[tag]["keys"][k])).float().double()
            for k in STATE6[tag]["params"]}


def test_wigner_l6_matches_reference_jd():
    """The closed-form harmonics' Wigner-D (oracle/e3nn_so3.py, any l <= 6) equals the reference's
    Jd.pt-based wigner_D (SO3_Rotation(6).set_wigner) block by block."""
    R = torch.from_numpy(Z6["wigner6/rot"])
    D = torch.from_numpy(Z6["wigner6/D"])
    np.testing.assert_allclose(EQ.wigner(R, 6).numpy(), D.numpy(), rtol=0, atol=1e-12)


def test_general_harmonics_reduce_to_the_explicit_ones():
    u = torch.nn.functional.normalize(torch.randn(40, 3, dtype=torch.float64), dim=-1)
    for l in range(3):
        np.testing.assert_allclose(E.sh_general(l, u).numpy(), E.sh_component(l, u).numpy(), rtol=0, atol=1e-14)


def test_grid_round_trip_exact_l6():
    for lmax in range(3, 7):
        rb, ra = 2 * (lmax + 1), 2 * (lmax + 1) + 1
        to, fr = E.ToS2Grid(lmax, (rb, ra), dtype=torch.float64), E.FromS2Grid((rb, ra), lmax, dtype=torch.float64)
        tm = torch.einsum("mbi,am->bai", to.shb, to.sha)
        fm = torch.einsum("am,mbi->bai", fr.sha, fr.shb)
        np.testing.assert_allclose(torch.einsum("bai,bak->ik", fm, tm).numpy(), np.eye((lmax + 1) ** 2), atol=1e-12)


def test_grid_matrices_l6_match_reference_construction():
    for l in range(7):
        for m in range(l + 1):
            to, fr = EQ.grid_mats(l, m)
            np.testing.assert_allclose(to.numpy(), Z6[f"grid/{l}{m}/to"], rtol=0, atol=1e-14)
            np.testing.assert_allclose(fr.numpy(), Z6[f"grid/{l}{m}/from"], rtol=0, atol=1e-14)


@pytest.mark.parametrize("tag", ["l6", "l4"])
def test_forward_lmax_gt2_matches_reference(tag):
    """The oracle at the reference's default degrees (lmax 6, mmax 2) and at lmax 4 / mmax 3 equals the
    reference model's own float64 forward (tests/golden/make_eqv2_l6.py)."""
    cfg = STATE6[tag]["config"]
    loc, vel, mass = Z6[f"{tag}/loc"], Z6[f"{tag}/vel"], Z6[f"{tag}/mass"]
    B, N = loc.shape[:2]
    acts = {}
    pred = EQ.forward(cfg, params6(tag), loc, vel, mass, B, N, Z6[f"{tag}/gauge"], acts=acts)
    np.testing.assert_allclose(pred.numpy(), Z6[f"{tag}/f64/pred"], rtol=1e-9, atol=1e-10)
    for k in ("edge_degree", "block0", "final_norm"):
        np.testing.assert_allclose(acts[k].numpy(), Z6[f"{tag}/f64/{k}"], rtol=1e-9, atol=1e-10)
