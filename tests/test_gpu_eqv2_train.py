"""EquiformerV2 training step on the device (trainer.py:233-358): the native operators
(csrc/eqv2_train.hip, nbx_eqv2_train_edges, and the GEMM / activation / LayerNorm / gather operators
shared with the SEGNN and PONITA steps) composed with autograd (eqv2_train.py) against torch fp64
autograd of the EquiformerV2 oracle (oracle/equiformer_v2.py, pinned to the reference model's own
outputs by tests/golden/eqv2.npz).

Tolerances (fp32 device arithmetic vs the fp64 oracle): operators 1e-5 relative of their scale
(gradients 1e-4); predictions per column 2e-5 * max|ref[:, c]| + 1e-7 (the EquiformerV2 forward's
stated tolerance); parameter gradients per tensor max|g - ref| <= 2e-4 * max|ref| + 1e-7."""
import numpy as np
import pytest
import torch

import nbody_amd.eqv2_train as T
from nbody_amd.equiformer_v2 import EquiformerV2_nbody
from nbody_amd.segnn_train import Graph as CSR
from oracle import equiformer_v2 as EQ
from oracle.graph import fc_edge_index

pytestmark = pytest.mark.gpu

SMALL = dict(num_layers=2, attn_hidden_channels=32, sphere_channels=32, num_heads=2, attn_alpha_channels=8,
             attn_value_channels=4, ffn_hidden_channels=32, lmax_list=[2], mmax_list=[1], edge_channels=32,
             num_distance_basis=64, max_neighbors=5, max_radius=4096.0)
C4 = dict(num_layers=4, attn_hidden_channels=64, sphere_channels=64, num_heads=4, attn_alpha_channels=8,
          attn_value_channels=4, ffn_hidden_channels=64, lmax_list=[2], mmax_list=[1], edge_channels=64,
          num_distance_basis=64, max_neighbors=5, max_radius=4096.0)


def _close(got, ref, rel, label):
    got = got.detach().double().cpu().numpy() if torch.is_tensor(got) else got
    ref = ref.detach().double().cpu().numpy() if torch.is_tensor(ref) else ref
    err = np.abs(got - ref).max()
    assert err <= rel * np.abs(ref).max() + 1e-7, (label, err, np.abs(ref).max())


@pytest.mark.parametrize("n0,nms,n_extra,cin,cout,E,radial,bias", [
    (3, (2,), 40, 128, 64, 1280, True, True),     # C4 so2_conv_1 (lmax 2 / mmax 1; extra = alpha + gating)
    (3, (2,), 0, 64, 16, 1280, False, True),      # C4 so2_conv_2 (no radial weights)
    (7, (6, 5), 9, 24, 20, 301, True, True),      # lmax 6 / mmax 2, ragged sizes
    (4, (3, 2, 1), 0, 12, 8, 77, True, False),    # lmax 3 / mmax 3, no bias
])
def test_so2_conv_matches_torch(hip_device, n0, nms, n_extra, cin, cout, E, radial, bias):
    """_SO2ConvFn (one grouped GEMM launch per direction; the complex pair product as one GEMM against
    [[Wr, -Wi], [Wi, Wr]]) vs fp64 torch autograd of SO2_Convolution's composition (so2_ops.py:78-156):
    outputs and the gradients of x, the radial weights, fc_m0 and every m > 0 fc."""
    from test_eqv2_train_host import _so2conv
    torch.manual_seed(E + cin)
    R = n0 + 2 * sum(nms)
    x = torch.randn(E, R, cin, dtype=torch.float64, requires_grad=True)
    rad = torch.randn(E, (n0 + sum(nms)) * cin, dtype=torch.float64, requires_grad=True) if radial else None
    W0 = torch.randn(n_extra + n0 * cout, n0 * cin, dtype=torch.float64, requires_grad=True)
    b0 = torch.randn(n_extra + n0 * cout, dtype=torch.float64, requires_grad=True) if bias else None
    Wm = [torch.randn(2 * nm * cout, nm * cin, dtype=torch.float64, requires_grad=True) for nm in nms]
    meta = (n0, tuple(nms), n_extra)
    out, extra = _so2conv(meta, x, rad, W0, b0, *Wm)
    go, ge = torch.randn_like(out), torch.randn_like(extra)
    ((out * go).sum() + (extra * ge).sum()).backward()
    dd = lambda t: t.detach().to(device=hip_device, dtype=torch.float32).contiguous().requires_grad_() \
        if t is not None else None
    xd, radd, W0d, b0d = dd(x), dd(rad), dd(W0), dd(b0)
    Wmd = [dd(w) for w in Wm]
    o, e = T._SO2ConvFn.apply(meta, xd, radd, W0d, b0d, *Wmd)
    cu = lambda t: t.to(hip_device, torch.float32)
    ((o * cu(go)).sum() + (e * cu(ge)).sum()).backward()
    _close(o, out, 1e-5, "out")
    if n_extra:
        _close(e, extra, 1e-5, "extra")
    _close(xd.grad, x.grad, 1e-5, "dx")
    if radial:
        _close(radd.grad, rad.grad, 1e-5, "drad")
    _close(W0d.grad, W0.grad, 1e-5, "dW0")
    if bias:
        _close(b0d.grad, b0.grad, 1e-5, "db0")
    for i, (g, r) in enumerate(zip(Wmd, Wm)):
        _close(g.grad, r.grad, 1e-5, f"dW{i + 1}")


@pytest.mark.parametrize("lmax,V,cin,cout", [(2, 320, 64, 64), (2, 37, 24, 40), (6, 23, 18, 33), (1, 5, 7, 3)])
def test_so3_linear_matches_torch(hip_device, lmax, V, cin, cout):
    """_SO3LinearFn (nbx_gemm_f32_grouped two-level rows, all degrees per launch) vs fp64 torch autograd
    of SO3_LinearV2 (so3.py:695-745: out[v][i] = W[l(i)] x[v][i], bias on i = 0): output, input, weight
    and bias gradients; ragged row counts, channel counts off the float4 path, lmax 6 (> 8 problems:
    two launches in the backward)."""
    torch.manual_seed(lmax * 100 + V)
    S = (lmax + 1) ** 2
    x = torch.randn(V, S, cin, dtype=torch.float64, requires_grad=True)
    W = torch.randn(lmax + 1, cout, cin, dtype=torch.float64, requires_grad=True)
    b = torch.randn(cout, dtype=torch.float64, requires_grad=True)
    deg = torch.tensor([l for l in range(lmax + 1) for _ in range(2 * l + 1)])
    ref = torch.einsum("vic,ioc->vio", x, W[deg]) + torch.cat([b[None], torch.zeros(S - 1, cout, dtype=torch.float64)])
    g = torch.randn_like(ref)
    (ref * g).sum().backward()
    dd = lambda t: t.detach().to(device=hip_device, dtype=torch.float32).contiguous().requires_grad_()
    xd, Wd, bd = dd(x), dd(W), dd(b)
    got = T._SO3LinearFn.apply(xd, Wd, bd, lmax)
    (got * g.to(hip_device, torch.float32)).sum().backward()
    _close(got, ref, 1e-5, "out")
    _close(xd.grad, x.grad, 1e-5, "dx")
    _close(Wd.grad, W.grad, 1e-5, "dW")
    _close(bd.grad, b.grad, 1e-5, "db")
    assert Wd.grad.is_contiguous() and Wd.grad.shape == W.shape


def test_rotation_s2_softmax_rmsnorm_match_torch(hip_device):
    """rotate / rotate_inv (adjoint pair), the S2 grid round trip, the segment softmax and the RMS norm:
    forward and input / parameter gradients vs fp64 torch autograd of the oracle's expressions."""
    torch.manual_seed(3)
    dev = hip_device
    B, N, C = 3, 5, 24
    V, E = B * N, B * N * (N - 1)
    dd = lambda x: x.detach().to(device=dev, dtype=torch.float32).contiguous().requires_grad_()
    # Wigner rows of random rotations (block diagonal, |m| <= 1 rows)
    R = torch.linalg.qr(torch.randn(E, 3, 3, dtype=torch.float64))[0]
    R = R * torch.sign(torch.linalg.det(R))[:, None, None]
    Dfull = EQ.wigner(R, 2)
    lay = EQ.Layout(2, 1)
    Dsel = Dfull[:, lay.sel, :].contiguous()
    x = torch.randn(E, 9, C, dtype=torch.float64, requires_grad=True)
    y = torch.randn(E, 7, C, dtype=torch.float64, requires_grad=True)
    ref_r = torch.bmm(Dsel, x)
    ref_i = torch.bmm(Dfull.transpose(1, 2)[:, :, lay.sel] * lay.rescale[None], y)
    dr, di = torch.randn_like(ref_r), torch.randn_like(ref_i)
    ((ref_r * dr).sum() + (ref_i * di).sum()).backward()
    D32 = Dsel.float().to(dev)
    xd, yd = dd(x), dd(y)
    got_r = T._RotateFn.apply(xd, D32, 0, 0)
    got_i = T._RotateFn.apply(yd, D32, 1, 1)
    ((got_r * dr.float().to(dev)).sum() + (got_i * di.float().to(dev)).sum()).backward()
    _close(got_r, ref_r, 1e-5, "rotate")
    _close(got_i, ref_i, 1e-5, "rotate_inv")
    _close(xd.grad, x.grad, 1e-5, "rotate adjoint")
    _close(yd.grad, y.grad, 1e-5, "rotate_inv adjoint")
    # S2 activation on both grids
    for lmax_m, I in ((1, 7), (2, 9)):
        to, fr = EQ.grid_mats(2, lmax_m)
        h = torch.randn(E, I, C, dtype=torch.float64, requires_grad=True)
        ref = EQ.Ctx.s2_act(h, (to, fr))
        dy = torch.randn_like(ref)
        (ref * dy).sum().backward()
        hd = dd(h)
        got = T._S2Fn.apply(hd, to.reshape(-1, I).float().to(dev), fr.reshape(-1, I).float().to(dev))
        (got * dy.float().to(dev)).sum().backward()
        _close(got, ref, 1e-5, f"s2 act I={I}")
        _close(hd.grad, h.grad, 1e-4, f"s2 act backward I={I}")
    # segment softmax over edge_index[1]
    ei = torch.as_tensor(fc_edge_index(B, N))
    g = CSR(ei, V, dev)
    lg = torch.randn(E, 3, dtype=torch.float64, requires_grad=True)
    mx = torch.full((V, 3), -np.inf, dtype=torch.float64).scatter_reduce(0, ei[1][:, None].expand(-1, 3), lg, "amax")
    ex = torch.exp(lg - mx[ei[1]])
    ref = ex / (torch.zeros(V, 3, dtype=torch.float64).index_add(0, ei[1], ex) + 1e-16)[ei[1]]
    da = torch.randn_like(ref)
    (ref * da).sum().backward()
    lgd = dd(lg)
    got = T._SoftmaxFn.apply(lgd, g)
    (got * da.float().to(dev)).sum().backward()
    _close(got, ref, 1e-5, "softmax")
    _close(lgd.grad, lg.grad, 1e-4, "softmax backward")
    # RMS norm over the spherical harmonics
    X = torch.randn(V, 9, C, dtype=torch.float64, requires_grad=True)
    w = torch.rand(3, C, dtype=torch.float64).add(0.5).requires_grad_()
    b = torch.randn(C, dtype=torch.float64, requires_grad=True)
    ref = EQ.rms_norm_sh({"n.affine_weight": w, "n.affine_bias": b}, "n", X, 2)
    dy = torch.randn_like(ref)
    (ref * dy).sum().backward()
    Xd, wd, bd = dd(X), dd(w), dd(b)
    got = T._RMSNormFn.apply(Xd, wd, bd, 1e-5)
    (got * dy.float().to(dev)).sum().backward()
    _close(got, ref, 1e-5, "rms norm")
    for name, a, r in (("dX", Xd, X), ("dw", wd, w), ("db", bd, b)):
        _close(a.grad, r.grad, 1e-4, "rms norm " + name)


def _model(cfg, device, seed=0, **kw):
    torch.manual_seed(seed)
    m = EquiformerV2_nbody(**cfg, alpha_drop=kw.pop("alpha_drop", 0.0), drop_path_rate=kw.pop("drop_path_rate", 0.0),
                           **kw)
    with torch.no_grad():     # non-trivial norms / biases / embeddings so that every gradient is exercised
        g = torch.Generator().manual_seed(seed + 1)
        for k, p in m.named_parameters():
            if k.endswith("bias") or "affine" in k or "norm" in k or "embedding.weight" in k:
                p.add_(0.1 * torch.randn(p.shape, generator=g))
    return m.to(device).train()


def _inputs(B, N, seed):
    rng = np.random.default_rng(seed)
    loc = rng.standard_normal((B, N, 3)) * 1.5
    vel = rng.standard_normal((B, N, 3)) * 0.3
    mass = rng.integers(1, 4, (B, N, 1)).astype(np.float64)
    gauge = rng.uniform(0, 1, (B * N * (N - 1), 3)).astype(np.float32)
    tgt = rng.standard_normal((B * N, 6)) * 0.1
    return loc, vel, mass, gauge, tgt


def _train_step(m, loc, vel, mass, gauge, tgt, device):
    B, N = loc.shape[:2]
    t = lambda a: torch.as_tensor(np.asarray(a), dtype=torch.float32, device=device).reshape(B * N, -1)
    batch = torch.arange(B, device=device).repeat_interleave(N)
    pos = t(loc)
    m.zero_grad(set_to_none=True)
    pred = m((pos, t(vel), torch.zeros_like(pos), t(mass), pos), batch,
             gauge=torch.as_tensor(gauge, dtype=torch.float32, device=device))
    loss = torch.nn.functional.mse_loss(pred, torch.as_tensor(tgt, dtype=pred.dtype, device=device))
    loss.backward()
    return float(loss.detach()), pred.detach().double().cpu().numpy(), {
        k: p.grad.double().cpu().numpy() for k, p in m.named_parameters() if p.grad is not None}


def _oracle(m, cfg, loc, vel, mass, gauge, tgt):
    B, N = loc.shape[:2]
    P = {k: p.detach().double().cpu().clone().requires_grad_() for k, p in m.named_parameters()}
    p32 = lambda a: np.asarray(a, np.float32).astype(np.float64)
    out = EQ.forward(cfg, P, p32(loc), p32(vel), mass, B, N, np.asarray(gauge, np.float64))
    loss = torch.nn.functional.mse_loss(out, torch.as_tensor(tgt))
    loss.backward()
    return float(loss.detach()), out.detach().numpy(), {k: v.grad.numpy() for k, v in P.items() if v.grad is not None}


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


@pytest.mark.parametrize("cfg,B,N", [(SMALL, 3, 5), (SMALL, 2, 8), (C4, 2, 20)], ids=["small-5", "small-8", "c4-20"])
def test_training_step_gradients_match_oracle(hip_device, cfg, B, N):
    """loss.backward() through the native operators: prediction, loss and every parameter gradient
    (embeddings, distance expansion, radial MLPs, SO(2) convolutions, attention norms / logits,
    projections, FFNs, RMS norms) vs fp64 autograd of the oracle, same gauges."""
    m = _model(cfg, hip_device)
    loc, vel, mass, gauge, tgt = _inputs(B, N, seed=B * 10 + N)
    rloss, rpred, rgrads = _oracle(m, cfg, loc, vel, mass, gauge, tgt)
    loss, pred, grads = _train_step(m, loc, vel, mass, gauge, tgt, hip_device)
    scale = np.abs(rpred).max(0)
    assert (np.abs(pred - rpred).max(0) <= 2e-5 * scale + 1e-7).all(), np.abs(pred - rpred).max(0) / scale
    assert abs(loss - rloss) <= 1e-5 * abs(rloss)
    worst = _check_grads(grads, rgrads)
    print(f"eqv2 B {B} N {N} C {cfg['sphere_channels']}: worst per-tensor gradient error {worst:.2e}")


def test_training_step_bit_reproducible_and_eval_matches_inference(hip_device):
    """Fixed-order reductions: bit-identical gradients over two backward passes.  An eval-mode
    grad forward (no dropout) equals the native inference forward on the same gauges."""
    B, N = 3, 6
    loc, vel, mass, gauge, tgt = _inputs(B, N, seed=4)
    runs = [_train_step(_model(SMALL, hip_device, seed=2), loc, vel, mass, gauge, tgt, hip_device) for _ in range(2)]
    for k in runs[0][2]:
        np.testing.assert_array_equal(runs[0][2][k], runs[1][2][k])
    m = _model(SMALL, hip_device, seed=2).eval()
    t = lambda a: torch.as_tensor(np.asarray(a), dtype=torch.float32, device=hip_device).reshape(B * N, -1)
    batch = torch.arange(B, device=hip_device).repeat_interleave(N)
    pos = t(loc)
    gg = torch.as_tensor(gauge, device=hip_device)
    with torch.no_grad():
        inf = m((pos, t(vel), torch.zeros_like(pos), t(mass), pos), batch, gauge=gg)
    m.native_train = True    # explicit: an eval-mode grad forward runs the training composition
    tr = m((pos, t(vel), torch.zeros_like(pos), t(mass), pos), batch, gauge=gg)
    assert tr.requires_grad
    torch.testing.assert_close(tr.detach(), inf, rtol=2e-5, atol=2e-6)


def test_training_with_dropout_and_adamw(hip_device):
    """The reference's training defaults (alpha_drop 0.1, drop_path_rate 0.05, train mode) with
    AdamW + clipping (trainer.py:170-194,309-321) on a fixed batch: finite, and the loss decreases."""
    B, N = 8, 5
    m = _model(SMALL, hip_device, seed=6, alpha_drop=0.1, drop_path_rate=0.05)
    loc, vel, mass, gauge, tgt = _inputs(B, N, seed=11)
    opt = torch.optim.AdamW(m.parameters(), lr=2e-3, weight_decay=1e-8)
    losses = []
    torch.manual_seed(0)
    for _ in range(25):
        loss, _, grads = _train_step(m, loc, vel, mass, gauge, tgt, hip_device)
        assert all(np.isfinite(g).all() for g in grads.values())
        torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
        opt.step()
        losses.append(loss)
    assert np.mean(losses[-5:]) < 0.8 * np.mean(losses[:5]), losses
