"""SEGNN training step on the device (trainer.py:233-358): the native training
operators (csrc/segnn_train.hip, include/nbx.h "SEGNN training step") composed with autograd
(segnn_train.py) against the torch fp64 autograd restatement of the reference forward
(oracle/segnn_torch.py, pinned to the numpy oracle in tests/test_oracle_segnn.py).

Tolerances (fp32 device arithmetic vs the fp64 oracle): operators to 1e-5 relative of their scale;
model predictions per column 1e-5 * max|ref[:, c]|; parameter gradients per tensor
max|g - ref| <= 2e-4 * max|ref| + 1e-7 (fp32 rounding accumulated through the six layers' backward;
measured ~1e-5)."""
import numpy as np
import pytest
import torch

import nbody_amd.graph as G
import nbody_amd.segnn as S
import nbody_amd.segnn_train as T
from nbody_amd import _lib
from oracle import segnn_torch as OT
from oracle.graph import fc_edge_index, knn_edge_index
from oracle.segnn import SEGNNOracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("flags", [0, 1, 2, 3])
@pytest.mark.parametrize("M,N,K,beta", [(70, 33, 45, 0.0), (130, 288, 386, 1.0), (96, 386, 5000, 0.0),
                                        (1, 1, 1, 0.0), (64, 64, 16, 1.0), (37, 5, 3000, 1.0)])
def test_gemm_f32_matches_torch(hip_device, flags, M, N, K, beta):
    """nbx_gemm_f32 in all four storage orders (split-K at the long-K shapes) vs fp64 torch."""
    g = torch.Generator().manual_seed(M * 7 + N + K)
    A = torch.randn(M, K, generator=g, dtype=torch.float64)
    B = torch.randn(K, N, generator=g, dtype=torch.float64)
    C0 = torch.randn(M, N, generator=g, dtype=torch.float64)
    ref = A @ B + beta * C0
    As = A.t().contiguous() if flags & 1 else A
    Bs = B.t().contiguous() if flags & 2 else B
    d = lambda x: x.to(device=hip_device, dtype=torch.float32).contiguous()
    C = d(C0)
    T.gemm(flags, M, N, K, d(As), As.shape[1], d(Bs), Bs.shape[1], C, N, beta)
    err = (C.double().cpu() - ref).abs().max().item()
    assert err <= 2e-6 * (A.abs() @ B.abs()).max().item() + 1e-6, err


@pytest.mark.parametrize("flags", [0, 1, 2, 3])
@pytest.mark.parametrize("M,N,K,ldb_pad", [(70, 34, 45, 0), (130, 289, 3840, 3), (96, 65, 1280, 0), (5, 1, 7, 1)])
def test_gemm_f32_ones_column(hip_device, flags, M, N, K, ldb_pad):
    """NBX_GEMM_B_ONES: op(B) [K][N - 1] from memory plus a last column of ones, so C's last column is the
    row sums of op(A) (the bias gradient of a weight-gradient GEMM); single and batched launches agree
    bit for bit, and the memory past op(B)'s N - 1 columns is never read."""
    g = torch.Generator().manual_seed(M + 3 * N + K)
    A = torch.randn(M, K, generator=g, dtype=torch.float64)
    B = torch.randn(K, N - 1, generator=g, dtype=torch.float64)
    ref = torch.cat([A @ B, A.sum(1, keepdim=True)], 1)
    As = A.t().contiguous() if flags & 1 else A
    # B stored with padding columns / rows filled with NaN: reading them would poison C
    Bs = B.t().contiguous() if flags & 2 else B
    ldb = Bs.shape[1] + ldb_pad
    Bp = torch.full((Bs.shape[0] + 1, ldb), float("nan"), dtype=torch.float64)
    Bp[:Bs.shape[0], :Bs.shape[1]] = Bs
    d = lambda x: x.to(device=hip_device, dtype=torch.float32).contiguous()
    Ad, Bd = d(As), d(Bp)
    C = torch.full((M, N), 7.0, device=hip_device)
    f = flags | _lib.GEMM_B_ONES
    T.gemm(f, M, N, K, Ad, As.shape[1], Bd, ldb, C, N)
    Cb = torch.full((M, N), 7.0, device=hip_device)
    T.gemm_batched([(f, M, N, K, Ad, As.shape[1], Bd, ldb, Cb, N, 0.0)])
    torch.cuda.synchronize()
    assert torch.isfinite(C).all()
    err = (C.double().cpu() - ref).abs().max().item()
    assert err <= 2e-6 * (A.abs() @ torch.cat([B.abs(), torch.ones(K, 1, dtype=torch.float64)], 1)).max().item() + 1e-6
    assert torch.equal(C, Cb)
    # NBX_GEMM_ONES_TAIL: the same result as one buffer [M][N - 1] (ldc = N - 1) + the row sums [M],
    # bit-identical to the column layout, single and batched; nothing past M N floats is written
    ft = f | _lib.GEMM_ONES_TAIL
    for batched in (False, True):
        Ct = torch.full((M * N + 5,), 7.0, device=hip_device)
        if batched:
            T.gemm_batched([(ft, M, N, K, Ad, As.shape[1], Bd, ldb, Ct, N - 1, 0.0)])
        else:
            T.gemm(ft, M, N, K, Ad, As.shape[1], Bd, ldb, Ct, N - 1)
        torch.cuda.synchronize()
        assert torch.equal(Ct[:M * (N - 1)].view(M, N - 1), C[:, :N - 1]), batched
        assert torch.equal(Ct[M * (N - 1):M * N], C[:, N - 1]), batched
        assert (Ct[M * N:] == 7.0).all(), batched


@pytest.mark.parametrize("M,N,K", [(320, 64, 64), (70, 33, 45), (96, 65, 1280), (5, 7, 3840)])
def test_gemm_f32_grouped_bias_and_two_level_rows(hip_device, M, N, K):
    """nbx_gemm_f32_grouped: the epilogue bias (unsplit and split-K shapes) equals the GEMM plus the bias
    added afterwards bit for bit, and two-level rows (rdiv 3 over an [M/3][5][K] array) equal the
    same rows copied out."""
    from nbody_amd.segnn_train import _at
    g = torch.Generator().manual_seed(M + N + K)
    d = lambda x: x.to(hip_device).contiguous()
    A, W, b = d(torch.randn(M, K, generator=g)), d(torch.randn(N, K, generator=g)), d(torch.randn(N, generator=g))
    C = torch.empty(M, N, device=hip_device)
    T.gemm_grouped([(_lib.GEMM_TRANS_B, M, N, K, _at(A, 0), K, _at(W, 0), K, _at(C, 0), N, 0.0, 1, 0, 0, 0,
                     _at(b, 0))], hip_device)
    C0 = torch.empty(M, N, device=hip_device)
    T.gemm_grouped([(_lib.GEMM_TRANS_B, M, N, K, _at(A, 0), K, _at(W, 0), K, _at(C0, 0), N, 0.0, 1, 0, 0, 0)],
                   hip_device)
    torch.cuda.synchronize()
    assert torch.equal(C, C0 + b)
    Mr = (M // 3) * 3
    if Mr:
        X = d(torch.randn(M // 3, 5, K, generator=g))          # rows 1..3 of every group of 5
        Y = torch.full((M // 3, 5, N), 7.0, device=hip_device)
        T.gemm_grouped([(_lib.GEMM_TRANS_B, Mr, N, K, _at(X, K), K, _at(W, 0), K, _at(Y, N), N, 0.0, 3, 5 * K, 0,
                         5 * N)], hip_device)
        Xc = X[:, 1:4].reshape(Mr, K).contiguous()
        Yc = torch.empty(Mr, N, device=hip_device)
        T.gemm_grouped([(_lib.GEMM_TRANS_B, Mr, N, K, _at(Xc, 0), K, _at(W, 0), K, _at(Yc, 0), N, 0.0, 1, 0, 0, 0)],
                       hip_device)
        torch.cuda.synchronize()
        assert torch.equal(Y[:, 1:4].reshape(Mr, N), Yc)
        assert (Y[:, 0] == 7.0).all() and (Y[:, 4] == 7.0).all()


@pytest.mark.parametrize("M,N,K,beta", [(8190, 160, 1000, 0.0), (8192, 128, 1024, 1.0), (4100, 452, 900, 0.0)])
def test_gemm_x3_large_products_match_fp64(hip_device, M, N, K, beta):
    """The bf16x3 kernel (gemm_x3_ok: C = A B^T on plain rows, >= 2^30 multiply-adds, K >= 64, N >= 96;
    tails in M, N and K) against fp64 torch at the fp32 kernels' bound, with the epilogue bias; one
    problem through nbx_gemm_f32 and the same problem in a two-problem nbx_gemm_f32_grouped launch agree
    bit for bit."""
    from nbody_amd.segnn_train import _at
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g, dtype=torch.float64)
    W = torch.randn(N, K, generator=g, dtype=torch.float64)
    b = torch.randn(N, generator=g, dtype=torch.float64)
    C0 = torch.randn(M, N, generator=g, dtype=torch.float64)
    d = lambda x: x.to(device=hip_device, dtype=torch.float32).contiguous()
    Ad, Wd, bd = d(A), d(W), d(b)
    bound = 2e-6 * (A.abs() @ W.abs().t()).max().item() + 1e-6
    C = d(C0)
    T.gemm(_lib.GEMM_TRANS_B, M, N, K, Ad, K, Wd, K, C, N, beta)
    ref = A @ W.t() + beta * C0
    assert (C.double().cpu() - ref).abs().max().item() <= bound
    Cg, C2 = d(C0), torch.empty(M, N, device=hip_device)
    T.gemm_grouped([(_lib.GEMM_TRANS_B, M, N, K, _at(Ad, 0), K, _at(Wd, 0), K, _at(Cg, 0), N, beta, 1, 0, 0, 0),
                    (_lib.GEMM_TRANS_B, M, N, K, _at(Ad, 0), K, _at(Wd, 0), K, _at(C2, 0), N, 0.0, 1, 0, 0, 0,
                     _at(bd, 0))], hip_device)
    torch.cuda.synchronize()
    assert torch.equal(Cg, C)
    assert (C2.double().cpu() - (A @ W.t() + b)).abs().max().item() <= bound


def test_gemm_f32_batched_equals_single(hip_device):
    """nbx_gemm_f32_batched (up to 4 GEMMs in one launch + one split-K sum launch) is bit-identical to
    nbx_gemm_f32 on each problem: mixed storage orders, split and unsplit shapes, beta 0 and 1."""
    g = torch.Generator().manual_seed(5)
    shapes = [(0, 320, 288, 386, 0.0), (1, 192, 386, 1280, 0.0), (2, 3840, 96, 192, 1.0), (3, 70, 33, 45, 0.0)]
    probs, singles = [], []
    for flags, M, N, K, beta in shapes:
        A = torch.randn(K, M, generator=g) if flags & 1 else torch.randn(M, K, generator=g)
        B = torch.randn(N, K, generator=g) if flags & 2 else torch.randn(K, N, generator=g)
        C0 = torch.randn(M, N, generator=g)
        d = lambda x: x.to(hip_device).contiguous()
        Ab, Bb = d(A), d(B)
        Cb, Cs = d(C0), d(C0)
        probs.append((flags, M, N, K, Ab, A.shape[1], Bb, B.shape[1], Cb, N, beta))
        T.gemm(flags, M, N, K, Ab, A.shape[1], Bb, B.shape[1], Cs, N, beta)
        singles.append(Cs)
    T.gemm_batched(probs)
    torch.cuda.synchronize()
    for p, cs in zip(probs, singles):
        assert torch.equal(p[8], cs)


def test_batchnorm_train_forward_backward(hip_device):
    """nbx_bn_train_forward / _backward vs autograd of the oracle's e3nn BatchNorm (batch stats)."""
    from oracle.e3nn_lite import Irreps
    rows, M = 777, 40
    rng = np.random.default_rng(3)
    s = rng.standard_normal((rows, M)) * 2 + 0.5
    v = rng.standard_normal((3, rows, M)) * 0.7
    w, b = rng.uniform(0.5, 1.5, 2 * M), rng.uniform(-0.3, 0.3, M)
    rm, rv = rng.uniform(-0.1, 0.1, M), rng.uniform(0.5, 1.5, 2 * M)
    dys, dyv = rng.standard_normal((rows, M)), rng.standard_normal((3, rows, M))
    # oracle (e3nn layout: M 0e channels then M 1o channels as xyz triples)
    x = torch.tensor(np.concatenate([s, v.transpose(1, 2, 0).reshape(rows, 3 * M)], 1), requires_grad=True)
    W, Bb = torch.tensor(w, requires_grad=True), torch.tensor(b, requires_grad=True)
    y, nrm, nrv = OT.batch_norm(x, Irreps(f"{M}x0e+{M}x1o"), W, Bb, torch.tensor(rm), torch.tensor(rv), True)
    dy = torch.tensor(np.concatenate([dys, dyv.transpose(1, 2, 0).reshape(rows, 3 * M)], 1))
    (y * dy).sum().backward()
    f = lambda a: torch.tensor(a, dtype=torch.float32, device=hip_device).contiguous()
    S_, V_, w_, b_, rm_, rv_ = f(s), f(v), f(w), f(b), f(rm), f(rv)
    OS, OV = T._BNFn.apply(S_.requires_grad_(), V_.requires_grad_(), w_.requires_grad_(), b_.requires_grad_(),
                           rm_, rv_, 1e-5, 0.1)
    (OS * f(dys)).sum().add((OV * f(dyv)).sum()).backward()
    yo = y.detach().numpy()
    np.testing.assert_allclose(OS.detach().cpu().numpy(), yo[:, :M], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(OV.detach().cpu().numpy(), yo[:, M:].reshape(rows, M, 3).transpose(2, 0, 1),
                               rtol=1e-5, atol=1e-5)
    gx = x.grad.numpy()
    np.testing.assert_allclose(S_.grad.cpu().numpy(), gx[:, :M], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(V_.grad.cpu().numpy(), gx[:, M:].reshape(rows, M, 3).transpose(2, 0, 1),
                               rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(w_.grad.cpu().numpy(), W.grad.numpy(), rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(b_.grad.cpu().numpy(), Bb.grad.numpy(), rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(rm_.cpu().numpy(), nrm.numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(rv_.cpu().numpy(), nrv.numpy(), rtol=1e-5, atol=1e-6)


def _model(hidden, layers, device, seed=0, perturb=True):
    torch.manual_seed(seed)
    m = S.SEGNN(hidden_features=hidden, num_layers=layers)
    if perturb:
        with torch.no_grad():
            for mod in m.modules():
                if isinstance(mod, S.BatchNorm):
                    mod.weight.uniform_(0.5, 1.5)
                    mod.bias.uniform_(-0.2, 0.2)
                    mod.running_mean.uniform_(-0.1, 0.1)
                    mod.running_var.uniform_(0.5, 1.5)
    return m.to(device).train()


def _inputs(B, N, seed):
    rng = np.random.default_rng(seed)
    pos = rng.standard_normal((B * N, 3)) * np.cbrt(N / 5)
    vel = rng.standard_normal((B * N, 3))
    mass = rng.uniform(0.5, 1.5, (B * N, 1))
    tgt = rng.standard_normal((B * N, 6)) * 0.3
    return pos, vel, mass, tgt


def _train_step(model, pos, vel, mass, ei, tgt, device, N=5):
    class Graph:
        pass
    g = Graph()
    t = lambda a: torch.tensor(a, dtype=torch.float32, device=device)
    g.pos, g.vel, g.mass = t(pos), t(vel), t(mass)
    g.edge_index = torch.as_tensor(np.asarray(ei), dtype=torch.int64, device=device)
    g.batch = torch.arange(pos.shape[0] // N, device=device).repeat_interleave(N)
    model.zero_grad(set_to_none=True)
    pred = model(g)
    loss = torch.nn.functional.mse_loss(pred, t(tgt))
    loss.backward()
    return float(loss), pred.detach().double().cpu().numpy(), {
        k: p.grad.double().cpu().numpy() for k, p in model.named_parameters() if p.grad is not None}


def _check_grads(got, ref, rel=2e-4):
    assert set(got) == set(ref), set(got) ^ set(ref)
    worst = 0.0
    gmax = max(np.abs(r).max() for r in ref.values())
    for k, r in ref.items():
        e = np.abs(got[k] - r).max()
        sc = np.abs(r).max()
        worst = max(worst, e / max(sc, 1e-6 * gmax))   # (some tensors' gradients vanish: absolute there)
        assert e <= rel * sc + 1e-7, (k, e, sc)
    return worst


def _oracle(model, hidden, layers, pos, vel, mass, ei, tgt):
    params = {k: v.double().cpu().numpy().copy() for k, v in model.state_dict().items() if "output_mask" not in k}
    om = SEGNNOracle(hidden_features=hidden, num_layers=layers)
    return OT.loss_and_grads(om, params, pos, vel, mass, ei, tgt)


@pytest.mark.parametrize("hidden,layers,B,N", [(16, 1, 3, 5), (32, 2, 4, 5), (24, 2, 3, 7), (192, 6, 8, 5)])
def test_training_step_gradients_match_oracle(hip_device, hidden, layers, B, N):
    """loss.backward() through the native training operators: prediction, loss, every parameter
    gradient (tensor products, biases, BatchNorm weight / bias) and the running statistics vs the
    torch fp64 autograd oracle; C2 widths (hidden 192, 6 layers) included."""
    model = _model(hidden, layers, hip_device)
    pos, vel, mass, tgt = _inputs(B, N, seed=hidden + layers)
    ei = fc_edge_index(B, N)
    rloss, rpred, rgrads, rstats = _oracle(model, hidden, layers, pos, vel, mass, ei, tgt)
    loss, pred, grads = _train_step(model, pos, vel, mass, ei, tgt, hip_device, N)
    scale = np.abs(rpred).max(0)
    assert (np.abs(pred - rpred).max(0) <= 1e-5 * scale + 1e-7).all(), np.abs(pred - rpred).max(0) / scale
    assert abs(loss - rloss) <= 1e-5 * abs(rloss)
    worst = _check_grads(grads, rgrads)
    print(f"hidden {hidden} layers {layers} B {B} N {N}: worst per-tensor gradient error {worst:.2e} (relative to max)")
    sd = model.state_dict()
    for k, v in rstats.items():
        np.testing.assert_allclose(sd[k].double().cpu().numpy(), v, rtol=1e-4, atol=1e-6)


def test_training_step_knn_graph(hip_device):
    """Training on build_graph_with_knn's kNN graph (num_neighbors=2 < N-1, the reference's SEGNN
    dataloader option, segnn_n_body_dataloader.py): gradients vs the oracle on the same edge_index."""
    hidden, layers, B, N = 32, 2, 6, 5
    model = _model(hidden, layers, hip_device, seed=4)
    pos, vel, mass, tgt = _inputs(B, N, seed=21)
    ei = knn_edge_index(pos.astype(np.float32).astype(np.float64), B, N, 2)
    p32 = lambda a: a.astype(np.float32).astype(np.float64)
    rloss, rpred, rgrads, _ = _oracle(model, hidden, layers, p32(pos), p32(vel), p32(mass), ei, tgt)
    loss, pred, grads = _train_step(model, pos, vel, mass, ei, tgt, hip_device)
    scale = np.abs(rpred).max(0)
    assert (np.abs(pred - rpred).max(0) <= 1e-5 * scale + 1e-7).all()
    _check_grads(grads, rgrads)


def test_training_step_bit_reproducible_and_float64_module(hip_device):
    """Fixed-order reductions: two backward passes give bit-identical gradients.  A float64 module
    (the reference's precision_mode: double) trains through the same fp32 operators: its gradients are
    float64 tensors equal to the fp32 module's."""
    hidden, layers, B, N = 32, 2, 5, 5
    pos, vel, mass, tgt = _inputs(B, N, seed=8)
    ei = fc_edge_index(B, N)
    runs = []
    for _ in range(2):
        model = _model(hidden, layers, hip_device, seed=2)
        runs.append(_train_step(model, pos, vel, mass, ei, tgt, hip_device)[2])
    for k in runs[0]:
        np.testing.assert_array_equal(runs[0][k], runs[1][k])
    m64 = _model(hidden, layers, hip_device, seed=2).double()
    _, _, g64 = _train_step(m64, pos, vel, mass, ei, tgt, hip_device)
    assert all(p.grad.dtype == torch.float64 for p in m64.parameters() if p.grad is not None)
    for k in runs[0]:
        np.testing.assert_allclose(g64[k], runs[0][k], rtol=1e-6, atol=1e-9)


def test_training_steps_with_adamw_decrease_loss(hip_device):
    """A few reference-style optimiser steps (AdamW + clipping, trainer.py:170-194,309-321) on a
    fixed batch lower the loss; the inference forward afterwards sees the updated weights."""
    model = _model(32, 2, hip_device, seed=5, perturb=False)
    B, N = 16, 5
    pos, vel, mass, tgt = _inputs(B, N, seed=9)
    ei = fc_edge_index(B, N)
    opt = torch.optim.AdamW(model.parameters(), lr=3e-3, weight_decay=1e-8, betas=(0.9, 0.98), eps=1e-9)
    losses = []
    for _ in range(12):
        loss, _, _ = _train_step(model, pos, vel, mass, ei, tgt, hip_device)
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        losses.append(loss)
    assert losses[-1] < 0.8 * losses[0], losses
    model.eval()

    class Graph:
        pass
    g = Graph()
    t = lambda a: torch.tensor(a, dtype=torch.float32, device=hip_device)
    g.pos, g.vel, g.mass, g.edge_index = t(pos), t(vel), t(mass), G.fc_edge_index(B, N, hip_device)
    with torch.no_grad():
        inf = model(g)
    model.native_train = True    # explicit: an eval-mode grad forward runs the training composition
    with torch.enable_grad():
        tr = model(g)       # eval-mode training forward: running statistics, same weights
    torch.testing.assert_close(inf, tr.detach(), rtol=1e-4, atol=1e-5)
