"""EquiformerV2 at general degrees on the device (lmax <= 6; the reference constructor's default
lmax_list = [6], mmax_list = [2]): the general-degree operators (csrc/eqv2_general.hip, the widened
nbx_eqv2_s2_act) and the composed forward / training step / rollout (eqv2_train.py) against

* the reference's own outputs: tests/golden/eqv2_l6.npz (make_eqv2_l6.py ran the reference model code:
  Wigner blocks of 16 frames from its Jd-based wigner_D, float64 forwards at lmax 6 / mmax 2 and
  lmax 4 / mmax 3);
* the float64 oracle (oracle/equiformer_v2.py, pinned to those fixtures by test_eqv2_oracle.py) with
  torch autograd for the gradients.

Tolerances (fp32 device arithmetic vs float64): operators 1e-5 of their scale (gradients 1e-4), Wigner
rows 2e-6 absolute (entries are <= 1); predictions per column 2e-5 * max|ref[:, c]| + 1e-7 (the
EquiformerV2 forward's stated tolerance); parameter gradients per tensor 2e-4 * max|ref| + 1e-7."""
import json
import os
import sys

import numpy as np
import pytest
import torch

import nbody_amd._lib as L
import nbody_amd.eqv2_train as T
from nbody_amd import so3
from nbody_amd.equiformer_v2 import EquiformerV2_nbody
from oracle import equiformer_v2 as EQ

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from eqv2_params import param_value  # noqa: E402

pytestmark = pytest.mark.gpu

Z6 = np.load(os.path.join(HERE, "golden", "eqv2_l6.npz"))
STATE6 = json.load(open(os.path.join(HERE, "golden", "eqv2_l6_state.json")))

L6 = dict(num_layers=2, attn_hidden_channels=32, sphere_channels=32, num_heads=2, attn_alpha_channels=8,
          attn_value_channels=4, ffn_hidden_channels=32, lmax_list=[6], mmax_list=[2], edge_channels=32,
          num_distance_basis=64, max_neighbors=5, max_radius=4096.0)
L3 = dict(L6, num_layers=1, sphere_channels=48, ffn_hidden_channels=40, lmax_list=[3], mmax_list=[3], num_heads=4)
SMALL2 = dict(L6, lmax_list=[2], mmax_list=[1])


def _dp(t):
    return L.dev_ptr(t)


def _st(dev):
    return L.stream_ptr(dev)


def _close(got, ref, rel, label, abs_=1e-7):
    got = got.detach().double().cpu().numpy() if torch.is_tensor(got) else np.asarray(got)
    ref = ref.detach().double().cpu().numpy() if torch.is_tensor(ref) else np.asarray(ref)
    err = np.abs(got - ref).max()
    assert err <= rel * np.abs(ref).max() + abs_, (label, err, np.abs(ref).max())
    return err


def _rotations(n, seed):
    g = torch.Generator().manual_seed(seed)
    R = torch.linalg.qr(torch.randn(n, 3, 3, dtype=torch.float64, generator=g))[0]
    return R * torch.sign(torch.linalg.det(R))[:, None, None]


def _wigner_rows(R, lmax, mmax, dev):
    """nbx_eqv2_wigner on frames R [E][3][3] -> dsel [E][S] (device)."""
    E = R.shape[0]
    lay = so3.Layout(lmax, mmax)
    rot = R.reshape(E, 9).float().to(dev).contiguous()
    tab = so3.wigner_table(lmax).to(dev)
    D = torch.empty(E, lay.dsel_floats, device=dev)
    L.check(L.lib().nbx_eqv2_wigner(E, lmax, mmax, _dp(rot), 9, _dp(tab), _dp(D), _st(dev)), "nbx_eqv2_wigner")
    return D


def _blocks(dsel, lmax, mmax):
    """dsel [E][S] -> dense kept rows [E][R][(lmax+1)^2] (host)."""
    lay = so3.Layout(lmax, mmax)
    d = dsel.double().cpu()
    out = torch.zeros(d.shape[0], lay.n_red, lay.n_full, dtype=torch.float64)
    off = roff = 0
    for l in range(lmax + 1):
        n, kl = 2 * l + 1, 2 * min(l, mmax) + 1
        out[:, roff:roff + kl, l * l:l * l + n] = d[:, off:off + kl * n].view(-1, kl, n)
        off, roff = off + kl * n, roff + kl
    return out


def test_wigner_rows_match_reference_jd(hip_device):
    """The kept rows of the reference's own Wigner blocks (SO3_Rotation(6).set_wigner, Jd.pt) for
    16 frames, at several mmax."""
    R = torch.from_numpy(Z6["wigner6/rot"])
    Dref = torch.from_numpy(Z6["wigner6/D"])
    for mmax in (0, 1, 2, 6):
        lay = so3.Layout(6, mmax)
        got = _blocks(_wigner_rows(R, 6, mmax, hip_device), 6, mmax)
        ref = Dref[:, lay.sel, :]
        err = (got - ref).abs().max().item()
        assert err <= 2e-6, (mmax, err)


@pytest.mark.parametrize("lmax,mmax", [(6, 2), (4, 3), (3, 0), (2, 1)])
def test_general_operators_match_torch(hip_device, lmax, mmax):
    """nbx_eqv2_wigner, rotate / rotate_inv (adjoint pair, rescale), the S2 round trip on
    SO3_Grid(lmax, mmax) and (lmax, lmax), and the RMS norm at C = 48 and 160: forward and gradients
    vs fp64 torch autograd of the oracle's expressions."""
    dev = hip_device
    torch.manual_seed(lmax * 10 + mmax)
    E, C = 40, 24
    dd = lambda x: x.detach().to(device=dev, dtype=torch.float32).contiguous().requires_grad_()
    lay, olay = so3.Layout(lmax, mmax), EQ.Layout(lmax, mmax)
    assert lay.sel == olay.sel and lay.perm == olay.perm
    R = _rotations(E, lmax)
    Dfull = EQ.wigner(R, lmax)
    D = _wigner_rows(R, lmax, mmax, dev)
    _close(_blocks(D, lmax, mmax), Dfull[:, lay.sel, :], 2e-6, "wigner rows")
    x = torch.randn(E, lay.n_full, C, dtype=torch.float64, requires_grad=True)
    y = torch.randn(E, lay.n_red, C, dtype=torch.float64, requires_grad=True)
    ref_r = torch.bmm(Dfull[:, lay.sel, :], x)
    ref_i = torch.bmm(Dfull.transpose(1, 2)[:, :, lay.sel] * olay.rescale[None], y)
    dr, di = torch.randn_like(ref_r), torch.randn_like(ref_i)
    ((ref_r * dr).sum() + (ref_i * di).sum()).backward()
    xd, yd = dd(x), dd(y)
    got_r = T._RotateGFn.apply(xd, D, lay, 0, 0)
    got_i = T._RotateGFn.apply(yd, D, lay, 1, 1)
    ((got_r * dr.float().to(dev)).sum() + (got_i * di.float().to(dev)).sum()).backward()
    _close(got_r, ref_r, 1e-5, "rotate")
    _close(got_i, ref_i, 1e-5, "rotate_inv")
    _close(xd.grad, x.grad, 1e-5, "rotate adjoint")
    _close(yd.grad, y.grad, 1e-5, "rotate_inv adjoint")
    # the m-primary row order of the SO(2) convolutions: rows permuted, values unchanged
    order = torch.tensor(lay.inv_perm, dtype=torch.int32, device=dev)
    perm = torch.tensor(lay.perm, device=dev)
    with torch.no_grad():
        torch.testing.assert_close(T._RotateGFn.apply(xd, D, lay, 0, 0, order), got_r[:, perm], rtol=0, atol=0)
        torch.testing.assert_close(T._RotateGFn.apply(yd[:, perm].contiguous(), D, lay, 1, 1, order), got_i,
                                   rtol=0, atol=0)
    for mm, I in ((mmax, lay.n_red), (lmax, lay.n_full)):
        to, fr = EQ.grid_mats(lmax, mm)
        h = torch.randn(E, I, C, dtype=torch.float64, requires_grad=True)
        ref = EQ.Ctx.s2_act(h, (to, fr))
        dy = torch.randn_like(ref)
        (ref * dy).sum().backward()
        hd = dd(h)
        got = T._S2Fn.apply(hd, to.reshape(-1, I).float().to(dev), fr.reshape(-1, I).float().to(dev))
        (got * dy.float().to(dev)).sum().backward()
        _close(got, ref, 1e-5, f"s2 act ({lmax}, {mm})")
        _close(hd.grad, h.grad, 1e-4, f"s2 act backward ({lmax}, {mm})")
    for Cn in (48, 160):
        X = torch.randn(30, lay.n_full, Cn, dtype=torch.float64, requires_grad=True)
        w = torch.rand(lmax + 1, Cn, dtype=torch.float64).add(0.5).requires_grad_()
        b = torch.randn(Cn, dtype=torch.float64, requires_grad=True)
        ref = EQ.rms_norm_sh({"n.affine_weight": w, "n.affine_bias": b}, "n", X, lmax)
        dy = torch.randn_like(ref)
        (ref * dy).sum().backward()
        Xd, wd, bd = dd(X), dd(w), dd(b)
        got = T._RMSNormGFn.apply(Xd, wd, bd, 1e-5, lmax)
        (got * dy.float().to(dev)).sum().backward()
        _close(got, ref, 1e-5, f"rms norm C={Cn}")
        for name, a, r in (("dX", Xd, X), ("dw", wd, w), ("db", bd, b)):
            _close(a.grad, r.grad, 1e-4, f"rms norm {name} C={Cn}")


@pytest.mark.parametrize("C", [8, 16, 32])
def test_rotate_small_channel_counts_stage_wigner_in_lds(hip_device, C):
    """rotate / rotate_inv at channel counts dividing the 256-thread block (the attention's nh nv = 16 at
    C4 widths): the block's Wigner blocks are staged in the LDS; E = 37 leaves a partial last block.
    Against fp64 torch, with the m-primary order and the inverse rescale."""
    dev, lmax, mmax, E = hip_device, 6, 2, 37
    lay, olay = so3.Layout(lmax, mmax), EQ.Layout(lmax, mmax)
    R = _rotations(E, 23)
    Dfull = EQ.wigner(R, lmax)
    D = _wigner_rows(R, lmax, mmax, dev)
    g = torch.Generator().manual_seed(C)
    x = torch.randn(E, lay.n_full, C, generator=g, dtype=torch.float64)
    y = torch.randn(E, lay.n_red, C, generator=g, dtype=torch.float64)
    order = torch.tensor(lay.inv_perm, dtype=torch.int32, device=dev)
    perm = torch.tensor(lay.perm)
    with torch.no_grad():
        got_r = T._RotateGFn.apply(x.float().to(dev), D, lay, 0, 0, order)
        got_i = T._RotateGFn.apply(y[:, perm].float().to(dev).contiguous(), D, lay, 1, 1, order)
    _close(got_r, torch.bmm(Dfull[:, lay.sel, :], x)[:, perm], 1e-5, f"rotate C={C}")
    _close(got_i, torch.bmm(Dfull.transpose(1, 2)[:, :, lay.sel] * olay.rescale[None], y), 1e-5,
           f"rotate_inv C={C}")


@pytest.mark.parametrize("C", [24, 64])
def test_rotate_gather_equals_gather_then_rotate(hip_device, C):
    """nbx_eqv2_rotate_gather (ABI 19; the attention's [x[src] | x[dst]] rotated without materialising
    it) is bit-identical to gather_pair followed by the rotation, forward and input gradient, on the
    m-primary row order, at C = 24 (per-lane Wigner reads) and C = 64 (wave-uniform edge, scalar
    reads: that rotation path is also checked against fp64 torch here)."""
    from nbody_amd.graph import fc_edge_index
    from nbody_amd.segnn_train import Graph
    dev = hip_device
    lmax, mmax, B, N = 6, 2, 2, 6
    V = B * N
    g = Graph(fc_edge_index(B, N, dev), V, dev)
    E = g.src.shape[0]
    lay = so3.Layout(lmax, mmax)
    R = _rotations(E, 17)
    D = _wigner_rows(R, lmax, mmax, dev)
    order = torch.tensor(lay.inv_perm, dtype=torch.int32, device=dev)
    X = torch.randn(V, lay.n_full, C, generator=torch.Generator().manual_seed(C), dtype=torch.float64)
    dy = torch.randn(E, lay.n_red, 2 * C, generator=torch.Generator().manual_seed(C + 1)).to(dev)
    xa = X.float().to(dev).requires_grad_()
    xb = X.float().to(dev).requires_grad_()
    fused = T._RotateGatherFn.apply(xa, g, D, lay, order)
    ref = T._RotateGFn.apply(T.gather_pair(xb, g), D, lay, 0, 0, order)
    (fused * dy).sum().backward()
    (ref * dy).sum().backward()
    torch.cuda.synchronize()
    assert torch.equal(fused, ref)
    assert torch.equal(xa.grad, xb.grad)
    src, dst = g.src.long().cpu(), g.dst.long().cpu()
    Dd = EQ.wigner(R, lmax)[:, lay.sel, :]
    want = torch.bmm(Dd, torch.cat([X[src], X[dst]], 2))[:, lay.perm]
    _close(fused, want, 1e-5, f"rotate gather C={C}")


def test_inference_radial_in_rotation_is_bit_identical(hip_device):
    """Under no_grad the attention applies SO2_Convolution's radial product in the gathered rotation's
    epilogue (rotate_gather_radial); in grad mode it stays a separate product.  Both round the same
    product once, so the lmax 6 fixture model's forward is bit-identical either way."""
    m = _fixture_model("l6", hip_device)
    loc, vel, mass = Z6["l6/loc"], Z6["l6/vel"], Z6["l6/mass"]
    B, N = loc.shape[:2]
    pos = _t(loc, B, N, hip_device)
    batch = torch.arange(B, device=hip_device).repeat_interleave(N)
    data = (pos, _t(vel, B, N, hip_device), torch.zeros_like(pos), _t(mass, B, N, hip_device), pos)
    gauge = torch.as_tensor(Z6["l6/gauge"], dtype=torch.float32, device=hip_device)
    with torch.no_grad():
        fused = m(data, batch, gauge=gauge)
    plain = m(data, batch, gauge=gauge)
    assert plain.requires_grad
    assert torch.equal(fused, plain.detach())


def _fixture_model(tag, device):
    torch.manual_seed(0)
    m = EquiformerV2_nbody(**STATE6[tag]["config"])
    with torch.no_grad():
        for k, p in m.named_parameters():
            p.copy_(torch.from_numpy(param_value(k, p.shape)).float())
    return m.to(device).eval()


def _t(a, B, N, device):
    return torch.as_tensor(np.asarray(a), dtype=torch.float32, device=device).reshape(B * N, -1)


@pytest.mark.parametrize("tag", ["l6", "l4"])
def test_forward_matches_reference_fixture(hip_device, tag):
    """The reference model's own float64 forward at lmax 6 / mmax 2 (its constructor default) and
    lmax 4 / mmax 3: the composed native path (no fused kernels exist for these degrees)."""
    from conftest import assert_cols
    m = _fixture_model(tag, hip_device)
    assert m._native_reason and m.uses_general_ops()
    loc, vel, mass = Z6[f"{tag}/loc"], Z6[f"{tag}/vel"], Z6[f"{tag}/mass"]
    B, N = loc.shape[:2]
    pos = _t(loc, B, N, hip_device)
    batch = torch.arange(B, device=hip_device).repeat_interleave(N)
    with torch.no_grad():
        out = m((pos, _t(vel, B, N, hip_device), torch.zeros_like(pos), _t(mass, B, N, hip_device), pos), batch,
                gauge=torch.as_tensor(Z6[f"{tag}/gauge"], dtype=torch.float32, device=hip_device))
    assert not out.requires_grad
    assert_cols(out.double().cpu().numpy(), Z6[f"{tag}/f64/pred"], rel=2e-5, label=f"eqv2 {tag} vs reference")


def _model(cfg, device, seed=0):
    torch.manual_seed(seed)
    m = EquiformerV2_nbody(**cfg, alpha_drop=0.0, drop_path_rate=0.0)
    with torch.no_grad():
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
    batch = torch.arange(B, device=device).repeat_interleave(N)
    pos = _t(loc, B, N, device)
    m.zero_grad(set_to_none=True)
    pred = m((pos, _t(vel, B, N, device), torch.zeros_like(pos), _t(mass, B, N, device), pos), batch,
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


@pytest.mark.parametrize("cfg,B,N", [(L6, 2, 5), (L3, 3, 4)], ids=["l6m2", "l3m3-c48"])
def test_training_step_gradients_match_oracle(hip_device, cfg, B, N):
    """loss.backward() through the general-degree operators: prediction, loss and every parameter
    gradient vs fp64 autograd of the oracle, same gauges."""
    m = _model(cfg, hip_device)
    loc, vel, mass, gauge, tgt = _inputs(B, N, seed=B * 10 + N)
    rloss, rpred, rgrads = _oracle(m, cfg, loc, vel, mass, gauge, tgt)
    loss, pred, grads = _train_step(m, loc, vel, mass, gauge, tgt, hip_device)
    scale = np.abs(rpred).max(0)
    assert (np.abs(pred - rpred).max(0) <= 2e-5 * scale + 1e-7).all(), np.abs(pred - rpred).max(0) / scale
    assert abs(loss - rloss) <= 1e-5 * abs(rloss)
    assert set(grads) == set(rgrads), set(grads) ^ set(rgrads)
    worst = 0.0
    for k, r in rgrads.items():
        e, sc = np.abs(grads[k] - r).max(), np.abs(r).max()
        worst = max(worst, e / max(sc, 1e-12))
        assert e <= 2e-4 * sc + 1e-7, (k, e, sc)
    print(f"eqv2 lmax {cfg['lmax_list'][0]} mmax {cfg['mmax_list'][0]}: worst gradient error {worst:.2e}")


def test_general_operators_at_lmax2_agree_with_the_specialised_ones(hip_device):
    """lmax 2 / mmax 1 through the general operators (the composed path's default) vs the specialised
    lmax-2 operators (specialised_ops = True) and the fused inference kernels, same weights and gauges."""
    B, N = 3, 6
    loc, vel, mass, gauge, tgt = _inputs(B, N, seed=11)
    ms = _model(SMALL2, hip_device, seed=5)
    ms.specialised_ops = True
    assert not ms.uses_general_ops()
    spec = _train_step(ms, loc, vel, mass, gauge, tgt, hip_device)
    mg = _model(SMALL2, hip_device, seed=5)
    assert mg.uses_general_ops()          # the default at lmax 2 / mmax 1 too
    gen = _train_step(mg, loc, vel, mass, gauge, tgt, hip_device)
    np.testing.assert_allclose(gen[1], spec[1], rtol=2e-5, atol=2e-6)
    for k, r in spec[2].items():
        assert np.abs(gen[2][k] - r).max() <= 1e-4 * np.abs(r).max() + 1e-7, k
    mg.eval()
    batch = torch.arange(B, device=hip_device).repeat_interleave(N)
    pos = _t(loc, B, N, hip_device)
    args = ((pos, _t(vel, B, N, hip_device), torch.zeros_like(pos), _t(mass, B, N, hip_device), pos), batch)
    gg = torch.as_tensor(gauge, device=hip_device)
    with torch.no_grad():
        fused = mg(*args, gauge=gg)                       # the fused kernels (configuration supported)
        composed = mg._composed(args[0][0], args[0][1], args[0][3].reshape(-1), B, N, gg, 0)
    torch.testing.assert_close(composed, fused, rtol=2e-5, atol=2e-6)


def _hash_uniform(seed, ctr):
    """csrc/eqv2.hip hash_uniform (splitmix64 finaliser) in numpy uint64."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + np.uint64(0x9E3779B97F4A7C15) * (ctr.astype(np.uint64) + np.uint64(1))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(40)).astype(np.float64) / 16777216.0


def test_composed_rollout_matches_oracle(hip_device):
    """Device self-feed at lmax 4 / mmax 3 (the composed path): 5 frames vs the float64 oracle's
    rollout with the device's gauge draws (frame f uses the counter of frame f - 1, as
    nbx_eqv2_rollout)."""
    tag = "l4"
    m = _fixture_model(tag, hip_device)
    cfg = STATE6[tag]["config"]
    loc, vel, mass = Z6[f"{tag}/loc"], Z6[f"{tag}/vel"], Z6[f"{tag}/mass"]
    B, N = loc.shape[:2]
    E, F, seed = B * N * (N - 1), 5, 1234
    f32 = lambda a: torch.as_tensor(np.asarray(a), dtype=torch.float32, device=hip_device)
    tp, tv = m.rollout(f32(loc), f32(vel), f32(mass), F, seed=seed)
    gauges = np.stack([_hash_uniform(seed, (f * E + np.arange(E))[:, None] * 3 + np.arange(3)).astype(np.float32)
                       for f in range(F - 1)]).astype(np.float64)
    p = {k: torch.from_numpy(param_value(k, STATE6[tag]["keys"][k])).float().double() for k in STATE6[tag]["params"]}
    p32 = lambda a: np.asarray(a, np.float32).astype(np.float64)
    rl, rv = EQ.rollout(cfg, p, p32(loc), p32(vel), mass, F, gauges)
    # per-frame scale-aware bound: fp32 rounding grows with the self-fed state
    for f in range(F):
        for got, ref in ((tp, rl), (tv, rv)):
            g, r = got[:, f].double().cpu().numpy(), ref[:, f].numpy()
            assert np.abs(g - r).max() <= 1e-4 * np.abs(r).max() * (f + 1), (f, np.abs(g - r).max())
