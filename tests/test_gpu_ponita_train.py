"""PONITA training step on the device (trainer.py:233-358): the native operators
(csrc/ponita_train.hip + the fp32 MFMA GEMM / column sums of csrc/segnn_train.hip, include/nbx.h
"PONITA training step") composed with autograd (ponita_train.py) against the torch fp64 autograd
restatement of the reference forward (oracle/ponita_torch.py, pinned to the numpy oracle, the
reference's golden vectors and finite differences in tests/test_oracle_ponita.py).

Tolerances (fp32 device arithmetic vs the fp64 oracle): operators to 1e-5 relative of their scale
(gradients 1e-4); model predictions per column 1e-5 * max|ref[:, c]| + 1e-7; parameter gradients
per tensor max|g - ref| <= 2e-4 * max|ref| + 1e-7 (the SEGNN training step's bound)."""
import numpy as np
import pytest
import torch

import nbody_amd.graph as G
import nbody_amd.ponita as P
import nbody_amd.ponita_train as T
from nbody_amd import _lib
from nbody_amd.segnn_train import Graph as CSR
from oracle import ponita_torch as OT
from oracle.graph import fc_edge_index, knn_edge_index

pytestmark = pytest.mark.gpu


def _d(a, dev):
    return torch.as_tensor(np.asarray(a), dtype=torch.float32, device=dev).contiguous()


def _close(got, ref, rel, label):
    got = got.detach().double().cpu().numpy() if torch.is_tensor(got) else got
    ref = ref.detach().double().cpu().numpy() if torch.is_tensor(ref) else ref
    err = np.abs(got - ref).max()
    assert err <= rel * np.abs(ref).max() + 1e-7, (label, err, np.abs(ref).max())


def test_featurize_matches_oracle_invariants(hip_device):
    B, N, O = 3, 6, 11
    rng = np.random.default_rng(0)
    pos, vel = rng.standard_normal((B * N, 3)), rng.standard_normal((B * N, 3))
    mass = rng.uniform(0.5, 1.5, B * N)
    grid = P.uniform_grid_s2(O).double()
    ei = fc_edge_index(B, N)
    g = CSR(torch.as_tensor(ei), B * N, hip_device)
    attr, fiber, lift = T.featurize(_d(pos, hip_device), _d(vel, hip_device), _d(mass, hip_device),
                                    _d(grid, hip_device), g)
    t = lambda a: torch.as_tensor(np.asarray(a), dtype=torch.float64)
    p32 = lambda a: t(np.asarray(a, dtype=np.float32))
    pos_, vel_, grid_ = p32(pos), p32(vel), p32(grid.numpy())
    a, fa = OT.invariants(grid_, pos_[ei[0]] - pos_[ei[1]])
    ref_attr = OT.poly_features(a).reshape(-1, 14)
    ref_fib = OT.poly_features(fa).reshape(-1, 3)
    _close(attr[:, :14], ref_attr, 1e-5, "attr")
    assert torch.count_nonzero(attr[:, 14:]) == 0
    _close(fiber[:, :3], ref_fib, 1e-6, "fiber")
    _close(lift[:, 0], np.repeat(np.asarray(mass, np.float32), O), 0, "lift mass")
    _close(lift[:, 1], (vel_ @ grid_.T).reshape(-1), 1e-6, "lift vel")


def test_operators_match_torch_autograd(hip_device):
    """Linear + bias + GELU, the spatial message, the fibre convolution and LayerNorm: forward and
    every input gradient vs fp64 torch autograd of the oracle's expressions."""
    torch.manual_seed(1)
    B, N, O, C = 4, 5, 7, 48
    V = B * N
    ei = torch.as_tensor(fc_edge_index(B, N))
    E = ei.shape[1]
    g = CSR(ei, V, hip_device)
    dd = lambda x: x.detach().to(device=hip_device, dtype=torch.float32).contiguous().requires_grad_()
    # linear (K = 14 inside a 16-wide row) + bias + GELU
    X = torch.randn(E * O, 16, dtype=torch.float64)
    X[:, 14:] = 0
    W, b = torch.randn(C, 14, dtype=torch.float64, requires_grad=True), torch.randn(C, dtype=torch.float64,
                                                                                   requires_grad=True)
    ref = OT.gelu(X[:, :14] @ W.T + b)
    dY = torch.randn_like(ref)
    (ref * dY).sum().backward()
    Wd, bd = dd(W), dd(b)
    got = T.linear(X.float().to(hip_device), Wd, bd, _lib.ACT_GELU, ldx=16)
    (got * dY.float().to(hip_device)).sum().backward()
    _close(got, ref, 1e-5, "linear")
    _close(Wd.grad, W.grad, 1e-4, "linear dW")
    _close(bd.grad, b.grad, 1e-4, "linear db")
    # message + fibre convolution + LayerNorm
    K = torch.randn(E * O, C, dtype=torch.float64, requires_grad=True)
    H = torch.randn(V * O, C, dtype=torch.float64, requires_grad=True)
    FK = torch.randn(O * O, C, dtype=torch.float64, requires_grad=True)
    bias = torch.randn(C, dtype=torch.float64, requires_grad=True)
    lw = torch.rand(C, dtype=torch.float64).add(0.5).requires_grad_()
    lb = torch.randn(C, dtype=torch.float64, requires_grad=True)
    x1 = torch.zeros(V, O, C, dtype=torch.float64).index_add(0, ei[1], K.view(E, O, C) * H.view(V, O, C)[ei[0]])
    x2 = torch.einsum("boc,opc->bpc", x1, FK.view(O, O, C)) / O + bias
    y = OT.layer_norm(x2, lw, lb).reshape(V * O, C)
    dY = torch.randn_like(y)
    (y * dY).sum().backward()
    Kd, Hd, FKd, bsd, lwd, lbd = dd(K), dd(H), dd(FK), dd(bias), dd(lw), dd(lb)
    x1d = T._MessageFn.apply(Kd, Hd, g, O)
    _close(x1d, x1.reshape(V * O, C), 1e-5, "message")
    x2d = T._FiberFn.apply(x1d, FKd, bsd, O)
    _close(x2d, x2.reshape(V * O, C), 1e-5, "fibre conv")
    yd = T._LayerNormFn.apply(x2d, lwd, lbd, 1e-5)
    _close(yd, y, 1e-5, "layer norm")
    (yd * dY.float().to(hip_device)).sum().backward()
    for name, a, r in (("dK", Kd, K), ("dH", Hd, H), ("dFK", FKd, FK), ("dbias", bsd, bias), ("dlnw", lwd, lw),
                       ("dlnb", lbd, lb)):
        _close(a.grad, r.grad, 1e-4, name)


def _model(hidden, layers, num_ori, device, seed=0, **kw):
    torch.manual_seed(seed)
    m = P.PONITA_NBODY(hidden_dim=hidden, layers=layers, num_ori=num_ori, **kw)
    m.model.materialize()
    return m.to(device).train()


def _inputs(B, N, seed):
    rng = np.random.default_rng(seed)
    pos = rng.standard_normal((B * N, 3)) * np.cbrt(N / 5)
    vel = rng.standard_normal((B * N, 3))
    mass = rng.uniform(0.5, 1.5, (B * N, 1))
    tgt = rng.standard_normal((B * N, 6)) * 0.3
    return pos, vel, mass, tgt


def _graph(pos, vel, mass, ei, device, N):
    class Gr:
        pass
    g = Gr()
    t = lambda a: torch.tensor(a, dtype=torch.float32, device=device)
    g.pos, g.vec, g.x = t(pos), t(vel).reshape(-1, 1, 3), t(mass)
    g.edge_index = torch.as_tensor(np.asarray(ei), dtype=torch.int64, device=device)
    g.rel_pos = g.pos[g.edge_index[0]] - g.pos[g.edge_index[1]]
    g.batch = torch.arange(pos.shape[0] // N, device=device).repeat_interleave(N)
    return g


def _train_step(model, pos, vel, mass, ei, tgt, device, N):
    g = _graph(pos, vel, mass, ei, device, N)
    model.zero_grad(set_to_none=True)
    pred = model(g)
    loss = torch.nn.functional.mse_loss(pred, torch.tensor(tgt, dtype=pred.dtype, device=device))
    loss.backward()
    return float(loss.detach()), pred.detach().double().cpu().numpy(), {
        k: p.grad.double().cpu().numpy() for k, p in model.named_parameters() if p.grad is not None}


def _calibrate(model, pos, vel, mass, ei, device, N):
    with torch.no_grad():
        model(_graph(pos, vel, mass, ei, device, N))
    assert all(bool(L.conv.callibrated) for L in model.model.interaction_layers)


def _check_grads(got, ref, rel=2e-4):
    assert set(got) == set(ref), set(got) ^ set(ref)
    worst = 0.0
    gmax = max(np.abs(r).max() for r in ref.values())
    for k, r in ref.items():
        e = np.abs(got[k] - r).max()
        sc = np.abs(r).max()
        worst = max(worst, e / max(sc, 1e-6 * gmax))
        assert e <= rel * sc + 1e-7, (k, e, sc)
    return worst


def _oracle(model, pos, vel, mass, ei, tgt):
    params = {k: v.double().cpu().numpy().copy() for k, v in model.state_dict().items()}
    p32 = lambda a: np.asarray(a, np.float32).astype(np.float64)
    return OT.loss_and_grads(params, model.model.ori_grid.double().cpu().numpy(), p32(pos), p32(vel), p32(mass),
                             ei, tgt, model.layers, multiple_readouts=model.multiple_readouts)


@pytest.mark.parametrize("hidden,layers,num_ori,B,N,kw", [
    (32, 2, 8, 3, 5, {"layer_scale": 0.3}),
    (64, 2, 12, 2, 9, {"layer_scale": 0.5, "multiple_readouts": False}),
    (32, 3, 6, 4, 4, {"layer_scale": 0.2, "basis_dim": 40}),
    (128, 8, 20, 4, 5, {}),                                  # the reference's training config (config.yaml)
])
def test_training_step_gradients_match_oracle(hip_device, hidden, layers, num_ori, B, N, kw):
    """loss.backward() through the native operators: prediction, loss and every parameter gradient
    (basis MLPs, embedding, conv kernels / bias, LayerNorm, ConvNext MLP, layer scale, read-outs) vs
    the torch fp64 autograd oracle, on the calibrated model the reference trains."""
    model = _model(hidden, layers, num_ori, hip_device, **kw)
    pos, vel, mass, tgt = _inputs(B, N, seed=hidden + layers)
    ei = fc_edge_index(B, N)
    _calibrate(model, pos, vel, mass, ei, hip_device, N)
    rloss, rpred, rgrads = _oracle(model, pos, vel, mass, ei, tgt)
    loss, pred, grads = _train_step(model, pos, vel, mass, ei, tgt, hip_device, N)
    scale = np.abs(rpred).max(0)
    assert (np.abs(pred - rpred).max(0) <= 1e-5 * scale + 1e-7).all(), np.abs(pred - rpred).max(0) / scale
    assert abs(loss - rloss) <= 1e-5 * abs(rloss)
    worst = _check_grads(grads, rgrads)
    print(f"hidden {hidden} layers {layers} O {num_ori} B {B} N {N}: worst per-tensor gradient error {worst:.2e}")


def test_training_step_knn_graph(hip_device):
    """Training on build_graph_with_knn's kNN graph (the reference's ponita_nbody dataloader option
    num_neighbors, ponita_n_body_dataloader.py:22-29): gradients vs the oracle on the same edge_index."""
    B, N = 5, 6
    model = _model(32, 2, 10, hip_device, seed=4, layer_scale=0.3)
    pos, vel, mass, tgt = _inputs(B, N, seed=21)
    ei = knn_edge_index(pos.astype(np.float32).astype(np.float64), B, N, 3)
    _calibrate(model, pos, vel, mass, ei, hip_device, N)
    rloss, rpred, rgrads = _oracle(model, pos, vel, mass, ei, tgt)
    loss, pred, grads = _train_step(model, pos, vel, mass, ei, tgt, hip_device, N)
    scale = np.abs(rpred).max(0)
    assert (np.abs(pred - rpred).max(0) <= 1e-5 * scale + 1e-7).all()
    _check_grads(grads, rgrads)


def test_first_grad_forward_calibrates_first(hip_device):
    """A fresh model's first grad-mode forward first performs the one-time calibration (the
    reference's train.py:49-77 no-grad dummy forward), then the training forward on the calibrated
    weights: the same weights as an explicit calibrating forward, the same gradients."""
    B, N = 3, 5
    pos, vel, mass, tgt = _inputs(B, N, seed=3)
    ei = fc_edge_index(B, N)
    a = _model(32, 2, 8, hip_device, seed=7, layer_scale=0.3)
    _calibrate(a, pos, vel, mass, ei, hip_device, N)
    _, pa, ga = _train_step(a, pos, vel, mass, ei, tgt, hip_device, N)
    b = _model(32, 2, 8, hip_device, seed=7, layer_scale=0.3)
    _, pb, gb = _train_step(b, pos, vel, mass, ei, tgt, hip_device, N)
    for (k, va), vb in zip(a.state_dict().items(), b.state_dict().values()):
        torch.testing.assert_close(va, vb, rtol=0, atol=0, msg=k)
    np.testing.assert_array_equal(pa, pb)
    for k in ga:
        np.testing.assert_array_equal(ga[k], gb[k])


def test_training_step_bit_reproducible_and_float64_module(hip_device):
    """Fixed-order reductions: two backward passes give bit-identical gradients.  A float64 module
    (the reference's ponita_nbody double_precision) trains through the same fp32 operators: its
    gradients are float64 tensors equal to the fp32 module's."""
    B, N = 4, 5
    pos, vel, mass, tgt = _inputs(B, N, seed=8)
    ei = fc_edge_index(B, N)
    runs = []
    for _ in range(2):
        model = _model(32, 2, 8, hip_device, seed=2, layer_scale=0.3)
        _calibrate(model, pos, vel, mass, ei, hip_device, N)
        runs.append(_train_step(model, pos, vel, mass, ei, tgt, hip_device, N)[2])
    for k in runs[0]:
        np.testing.assert_array_equal(runs[0][k], runs[1][k])
    m64 = _model(32, 2, 8, hip_device, seed=2, layer_scale=0.3)
    _calibrate(m64, pos, vel, mass, ei, hip_device, N)
    m64 = m64.double()
    _, _, g64 = _train_step(m64, pos, vel, mass, ei, tgt, hip_device, N)
    assert all(p.grad.dtype == torch.float64 for p in m64.parameters() if p.grad is not None)
    for k in runs[0]:
        np.testing.assert_allclose(g64[k], runs[0][k], rtol=1e-5, atol=1e-9)


def test_training_steps_with_adamw_track_oracle(hip_device):
    """Reference-style optimiser steps (AdamW + clipping, trainer.py:170-194,309-321) on a fixed batch:
    the device loss trajectory tracks the same steps taken on the fp64 oracle's gradients (relative
    1e-3 over 20 steps) and decreases; the inference forward afterwards sees the updated weights."""
    B, N, steps = 16, 5, 20
    model = _model(64, 2, 12, hip_device, seed=5, layer_scale=0.1)
    pos, vel, mass, tgt = _inputs(B, N, seed=9)
    ei = fc_edge_index(B, N)
    _calibrate(model, pos, vel, mass, ei, hip_device, N)
    # the oracle's trajectory from the same calibrated weights
    Pc = {k: torch.tensor(v.double().cpu().numpy(), requires_grad=not (k.endswith("callibrated") or
                                                                     k.endswith("ori_grid")))
          for k, v in model.state_dict().items()}
    learn = [v for v in Pc.values() if v.requires_grad]
    optc = torch.optim.AdamW(learn, lr=3e-3, weight_decay=1e-5)
    p32 = lambda a: torch.tensor(np.asarray(a, np.float32), dtype=torch.float64)
    pc, vc, mc, tc = p32(pos), p32(vel)[:, None], p32(mass), torch.tensor(tgt)
    eic = torch.as_tensor(ei)
    ref = []
    for _ in range(steps):
        optc.zero_grad()
        lc = torch.nn.functional.mse_loss(OT.forward(Pc, mc, vc, eic, pc[eic[0]] - pc[eic[1]], Pc["model.ori_grid"],
                                                     2), tc)
        lc.backward()
        torch.nn.utils.clip_grad_norm_(learn, 1.0)
        optc.step()
        ref.append(float(lc.detach()))
    opt = torch.optim.AdamW(model.parameters(), lr=3e-3, weight_decay=1e-5)
    losses = []
    for _ in range(steps):
        loss, _, _ = _train_step(model, pos, vel, mass, ei, tgt, hip_device, N)
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        losses.append(loss)
    np.testing.assert_allclose(losses, ref, rtol=1e-3)
    assert losses[-1] < 0.85 * losses[0], losses
    g = _graph(pos, vel, mass, ei, hip_device, N)
    g.edge_index = G.fc_edge_index(B, N, hip_device)
    with torch.no_grad():
        inf = model(g)
    with torch.enable_grad():
        tr = model(g)
    torch.testing.assert_close(inf, tr.detach(), rtol=1e-4, atol=1e-5)
