"""Known-answer tests that pin the SEGNN oracle's e3nn restatement (parity vs
e3nn itself is unpinned: e3nn 0.5.1 is not installable here)."""
import math

import numpy as np
import pytest

from oracle import e3nn_lite as e3
from oracle.graph import fc_edge_index
from oracle.segnn import SEGNNOracle, init_params, o3_transform, weight_balanced_irreps


def test_param_count_c2():
    # hidden=192, lmax_h=1, 6 layers -> 1,947,552 parameters
    m = SEGNNOracle(hidden_features=192, num_layers=6)
    assert str(m.hidden_irreps) == "96x0e+96x1o"
    assert m.num_params() == 1_947_552
    expect = {"embedding": (576, 96), "ml1": (111168, 192), "ml2": (55296, 192), "ul1": (110592, 192),
              "ul2": (36864, 96), "pre_pool1": (55296, 192), "pre_pool2": (384, 0)}
    for name, (nw, nb) in expect.items():
        t = getattr(m, name)
        assert (t.tp.weight_numel, len(t.bias_idx)) == (nw, nb), name


@pytest.mark.parametrize("H", [2, 7, 64, 96, 128, 192])
def test_weight_balanced_irreps(H):
    ir = weight_balanced_irreps(H, e3.Irreps("1x0e+1x1o"), 1)
    n = math.ceil(H / 2)
    assert str(ir) == f"{n}x0e+{n}x1o"


def test_normalize2mom_constants():
    import torch
    assert abs(e3.normalize2mom_constant(torch.nn.functional.silu) - e3.C_SILU) < 1e-12
    assert abs(e3.normalize2mom_constant(torch.sigmoid) - e3.C_SIGMOID) < 1e-12


def test_wigner_frobenius_normalised():
    for ls in [(0, 0, 0), (0, 1, 1), (1, 0, 1), (1, 1, 0), (1, 1, 1)]:
        assert abs(np.linalg.norm(e3.wigner_3j(*ls)) - 1) < 1e-14


def test_closed_form_paths():
    rng = np.random.default_rng(0)
    # 1x1o (x) 1x1o -> 1x0e : coefficient sqrt(1/1), CG = delta/sqrt3  -> w * x.y / sqrt3
    tp = e3.FullyConnectedTP("1x1o", "1x1o", "1x0e")
    x, y, w = rng.standard_normal((4, 3)), rng.standard_normal((4, 3)), rng.standard_normal(1)
    np.testing.assert_allclose(tp(x, y, w)[:, 0], w[0] * (x * y).sum(1) / math.sqrt(3), rtol=1e-13)
    # 2x0e (x) 1x1o -> 1x1o : fan_in 2, coefficient sqrt(3/2), CG = delta/sqrt3 -> sum_u w_u x_u y / sqrt2
    tp = e3.FullyConnectedTP("2x0e", "1x1o", "1x1o")
    x, y, w = rng.standard_normal((4, 2)), rng.standard_normal((4, 3)), rng.standard_normal(2)
    np.testing.assert_allclose(tp(x, y, w), (x @ w)[:, None] * y / math.sqrt(2), rtol=1e-13)
    # spherical harmonics l<=1, integral normalisation
    v = np.array([[3.0, 0.0, 4.0]])
    np.testing.assert_allclose(e3.spherical_harmonics_l1(v), [[e3.SH_C0, e3.SH_C1 * 0.6, 0.0, e3.SH_C1 * 0.8]])


def _random_rotation(rng):
    q, _ = np.linalg.qr(rng.standard_normal((3, 3)))
    return q * np.sign(np.linalg.det(q))


def test_segnn_oracle_equivariance():
    """Model-level E(3) equivariance (the featurisation's pos.mean over xyz is a
    reference quirk that is not equivariant, so rotate the featurised inputs)."""
    rng = np.random.default_rng(1)
    B, N = 3, 5
    m = SEGNNOracle(hidden_features=16, num_layers=2)
    p = init_params(m, seed=3)
    pos, vel, mass = rng.standard_normal((B * N, 3)), rng.standard_normal((B * N, 3)), np.ones((B * N, 1))
    ei = fc_edge_index(B, N)
    R = _random_rotation(rng)

    def feats(pos, vel):
        x, ea, na, amf = o3_transform(pos, vel, mass, ei)
        x[:, 0:3] = pos - pos.mean(0, keepdims=True)   # equivariant stand-in for the quirky centring
        return x, ea, na, amf

    x, ea, na, amf = feats(pos, vel)
    out, _ = m.forward(dict(p), x, ei, ea, na, amf)
    xr, ear, nar, amfr = feats(pos @ R.T, vel @ R.T)
    out_r, _ = m.forward(dict(p), xr, ei, ear, nar, amfr)
    np.testing.assert_allclose(out_r[:, :3], out[:, :3] @ R.T, atol=1e-10)
    np.testing.assert_allclose(out_r[:, 3:], out[:, 3:] @ R.T, atol=1e-10)


def test_batchnorm_train_and_eval():
    rng = np.random.default_rng(2)
    ir = e3.Irreps("3x0e+2x1o")
    x = rng.standard_normal((50, ir.dim))
    w, b = rng.uniform(0.5, 2, 5), rng.standard_normal(3)
    y, rm, rv = e3.batch_norm(x, ir, w, b, np.zeros(3), np.ones(5), training=True)
    s = x[:, :3]
    np.testing.assert_allclose(y[:, :3], (s - s.mean(0)) / np.sqrt(s.var(0) + 1e-5) * w[:3] + b, rtol=1e-12)
    v = x[:, 3:].reshape(50, 2, 3)
    n = (v ** 2).mean(2).mean(0)
    np.testing.assert_allclose(y[:, 3:].reshape(50, 2, 3), v / np.sqrt(n + 1e-5)[None, :, None] * w[3:, None],
                               rtol=1e-12)
    np.testing.assert_allclose(rm, 0.1 * s.mean(0))
    np.testing.assert_allclose(rv, 0.9 + 0.1 * np.concatenate([s.var(0), n]))
    ye, _, _ = e3.batch_norm(x, ir, w, b, rm, rv, training=False)
    np.testing.assert_allclose(ye[:, :3], (s - rm) / np.sqrt(rv[:3] + 1e-5) * w[:3] + b, rtol=1e-12)


def test_torch_oracle_matches_numpy_oracle():
    """oracle/segnn_torch.py (the autograd reference of the training step) is the numpy oracle's
    forward in torch: predictions and running statistics agree to fp64 rounding on fully-connected
    and kNN graphs, and its gradients match central finite differences of the numpy oracle's loss."""
    import torch
    from oracle import segnn_torch as ST
    from oracle.graph import fc_edge_index, knn_edge_index
    from oracle.segnn import SEGNNOracle, init_params, o3_transform
    om = SEGNNOracle(hidden_features=16, num_layers=2)
    p = init_params(om, 1)
    rng = np.random.default_rng(0)
    B, N = 3, 5
    pos, vel = rng.standard_normal((B * N, 3)), rng.standard_normal((B * N, 3))
    mass = rng.uniform(0.5, 1.5, (B * N, 1))
    for ei in (fc_edge_index(B, N), knn_edge_index(pos, B, N, 2)):
        x, ea, na, amf = o3_transform(pos, vel, mass, ei)
        ref, st = om.forward(p, x, ei, ea, na, amf, training=True)
        P = {k: torch.tensor(v) for k, v in p.items()}
        out, st2 = ST.forward(om, P, torch.tensor(pos), torch.tensor(vel), torch.tensor(mass), torch.tensor(ei), True)
        np.testing.assert_allclose(out.numpy(), ref, rtol=1e-12, atol=1e-13)
        for k in st:
            np.testing.assert_allclose(st2[k].numpy(), st[k], rtol=1e-12, atol=1e-13)
    # gradients vs finite differences of the numpy oracle's MSE loss, a few entries per kind
    ei = fc_edge_index(B, N)
    tgt = rng.standard_normal((B * N, 6))
    _, _, grads, _ = ST.loss_and_grads(om, p, pos, vel, mass, ei, tgt)
    x, ea, na, amf = o3_transform(pos, vel, mass, ei)

    def loss(q):
        return float(((om.forward(q, x, ei, ea, na, amf, training=True)[0] - tgt) ** 2).mean())
    for key in ("layers.0.message_layer_1.tp.weight", "layers.1.update_layer_2.biases",
                "layers.0.message_norm.weight", "layers.1.feature_norm.bias", "pre_pool2.tp.weight",
                "embedding_layer.tp.weight"):
        for j in (0, len(p[key]) // 2, len(p[key]) - 1):
            h = 1e-6
            qp, qm = dict(p), dict(p)
            qp[key], qm[key] = p[key].copy(), p[key].copy()
            qp[key][j] += h
            qm[key][j] -= h
            fd = (loss(qp) - loss(qm)) / (2 * h)
            assert abs(fd - grads[key][j]) <= 1e-6 * max(1.0, abs(fd)), (key, j, fd, grads[key][j])
