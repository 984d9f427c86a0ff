"""CPU check of the EquiformerV2 training composition (eqv2_train.py, host logic): with every native
operator swapped for its torch definition (fp64), ``train_forward`` equals the oracle
(oracle/equiformer_v2.py) given the same S2 grid matrices, and its autograd gradients equal the
oracle's.  The native operators themselves are checked on the GPU (tests/test_gpu_eqv2_train.py)."""
import numpy as np
import pytest
import torch

import nbody_amd.eqv2_train as T
from nbody_amd.equiformer_v2 import EquiformerV2_nbody
from oracle import equiformer_v2 as EQ

CFG = dict(num_layers=2, attn_hidden_channels=32, sphere_channels=32, num_heads=2, attn_alpha_channels=8,
           attn_value_channels=4, ffn_hidden_channels=32, lmax_list=[2], mmax_list=[1], edge_channels=32,
           num_distance_basis=64, max_neighbors=5, max_radius=4096.0)


class _G:
    def __init__(self, ei, V):
        self.src, self.dst, self.V, self.E = ei[0].long(), ei[1].long(), V, ei.shape[1]
        self.sptr = self.seid = self.dptr = self.deid = None


def _lin(X, W, b=None, act=0, ldx=None):
    y = X[:, :W.shape[1]] @ W.T      # ldx > K: the first K columns of each row (the operator's lda)
    return _act(y + b if b is not None else y, act)


def _act(X, k):
    if k == 2:
        return X * torch.sigmoid(X)
    if k == 3:
        return 0.6 * X + 0.4 * X * (2 * torch.sigmoid(X) - 1)
    assert k == 0
    return X


def _fn(f):
    return type("F", (), {"apply": staticmethod(f)})


def _so2conv(meta, x, rad, W0, b0, *Wm):
    """SO2_Convolution (so2_ops.py:78-156) on m-primary rows, as torch ops: m = 0 block through fc_m0,
    each m > 0 pair (+m, -m) through fc as the complex product (xr[+m] - xi[-m], xr[-m] + xi[+m])."""
    n0, nms, n_extra = meta
    E, R, cin = x.shape
    parts = torch.split(x, [n0] + [2 * nm for nm in nms], 1)
    rparts = torch.split(rad, [n0 * cin] + [nm * cin for nm in nms], 1) if rad is not None else None
    x0 = parts[0].reshape(E, n0 * cin)
    if rad is not None:
        x0 = x0 * rparts[0]
    y0 = x0 @ W0.T + (b0 if b0 is not None else 0.0)
    extra, y0 = y0[:, :n_extra], y0[:, n_extra:]
    cout = y0.shape[1] // n0
    outs = [y0.reshape(E, n0, cout)]
    sign = torch.tensor([-1.0, 1.0], dtype=x.dtype, device=x.device).view(1, 2, 1)
    for i, nm in enumerate(nms):
        xmm = parts[i + 1].reshape(E, 2, nm * cin)
        if rad is not None:
            xmm = xmm * rparts[i + 1][:, None]
        y = (xmm.reshape(2 * E, nm * cin) @ Wm[i].T).view(E, 2, 2, nm * cout)
        xr, xi = y.unbind(2)
        outs.append((xr + xi.flip(1) * sign).reshape(E, 2 * nm, cout))
    return torch.cat(outs, 1), extra


def _so3_linear(X, W, b, lmax):
    """SO3_LinearV2 (so3.py:695-745): per-degree weight, bias on the l = 0 row."""
    deg = torch.tensor([l for l in range(lmax + 1) for _ in range(2 * l + 1)])
    y = torch.einsum("vic,ioc->vio", X, W[deg])
    return torch.cat([y[:, :1] + b, y[:, 1:]], 1) if b is not None else y


def _rotate(X, D, inverse, rescale):
    if not inverse:
        return torch.bmm(D, X)
    return torch.bmm(D.transpose(1, 2) * (EQ.Layout(2, 1).rescale[None] if rescale else 1.0), X)


def _rotate_general(X, D, lay, inverse, rescale, order=None):
    """nbx_eqv2_rotate_general on dense kept rows D [E][R][(lmax+1)^2]; the [E][R] side's row of kept
    coefficient k is order[k] (None: k)."""
    if not inverse:
        y = torch.bmm(D, X)
        if order is not None:
            out = torch.empty_like(y)
            out[:, order.long()] = y
            return out
        return y
    if order is not None:
        X = X[:, order.long()]
    return torch.bmm(D.transpose(1, 2) * (EQ.Layout(lay.lmax, lay.mmax).rescale[None] if rescale else 1.0), X)


def _s2(X, Tm, Fm):
    t = torch.einsum("pi,zic->zpc", Tm, X)
    return torch.einsum("pi,zpc->zic", Fm, t * torch.sigmoid(t))


def _softmax(lg, g):
    nh = lg.shape[1]
    mx = torch.full((g.V, nh), -np.inf, dtype=lg.dtype).scatter_reduce(0, g.dst[:, None].expand(-1, nh), lg, "amax")
    ex = torch.exp(lg - mx[g.dst])
    return ex / (torch.zeros(g.V, nh, dtype=lg.dtype).index_add(0, g.dst, ex) + 1e-16)[g.dst]


@pytest.fixture
def torch_ops(monkeypatch):
    monkeypatch.setattr(T, "_f32", torch.float64)
    monkeypatch.setattr(T, "_f", lambda t: t.double())
    monkeypatch.setattr(T, "gather", lambda X, g, w: X[g.src if w == "s" else g.dst])
    monkeypatch.setattr(T, "gather_pair", lambda X, g: torch.cat([X[g.src], X[g.dst]], 2))
    monkeypatch.setattr(T, "linear", _lin)
    monkeypatch.setattr(T, "act", _act)
    monkeypatch.setattr(T, "_LayerNormFn", _fn(lambda X, w, b, eps: EQ.layer_norm(X, w, b, eps)))
    monkeypatch.setattr(T, "_SO3LinearFn", _fn(_so3_linear))
    monkeypatch.setattr(T, "_SO2ConvFn", _fn(_so2conv))
    monkeypatch.setattr(T, "_RotateFn", _fn(_rotate))
    monkeypatch.setattr(T, "_S2Fn", _fn(_s2))
    monkeypatch.setattr(T, "_SoftmaxFn", _fn(_softmax))
    monkeypatch.setattr(T, "_RMSNormFn", _fn(lambda X, w, b, eps: EQ.rms_norm_sh(
        {"n.affine_weight": w, "n.affine_bias": b}, "n", X, 2, eps)))
    monkeypatch.setattr(T, "_RotateGFn", _fn(_rotate_general))
    monkeypatch.setattr(T, "_RotateGatherFn", _fn(lambda X, g, D, lay, order: _rotate_general(
        torch.cat([X[g.src], X[g.dst]], 2), D, lay, 0, 0, order)))
    monkeypatch.setattr(T, "rotate_gather_radial", lambda X, g, D, lay, order, rad, radrow: _rotate_general(
        torch.cat([X[g.src], X[g.dst]], 2), D, lay, 0, 0, order) * rad.view(rad.shape[0], -1, 2 * X.shape[2])[
        :, radrow.long()])
    monkeypatch.setattr(T, "_RMSNormGFn", _fn(lambda X, w, b, eps, lmax: EQ.rms_norm_sh(
        {"n.affine_weight": w, "n.affine_bias": b}, "n", X, lmax, eps)))
    monkeypatch.setattr(T, "_SegSumFn", _fn(lambda X, idx, p, e, V: torch.zeros(V, X.shape[1], dtype=X.dtype)
                                             .index_add(0, idx.long(), X)))

    def step_init(self, model, pos, vel, charges, B, N, gauge, seed, frame=0):
        self.m, self.B, self.N, self.V, self.E = model, B, N, B * N, B * N * (N - 1)
        lay = self.lay = model.layout
        self.general = model.uses_general_ops()
        cfg = dict(lmax_list=model.lmax_list, mmax_list=model.mmax_list)
        ctx = EQ.Ctx(cfg, dict(model.state_dict()), pos, vel, charges, B, N, gauge)
        self.D = ctx.D[:, EQ.Layout(lay.lmax, lay.mmax).sel, :]
        self.perm, self.inv_perm, self.m0 = (torch.tensor(v) for v in (lay.perm, lay.inv_perm, lay.m0))
        self.order = torch.tensor(lay.inv_perm, dtype=torch.int32)
        self.sign = torch.tensor([-1.0, 1.0], dtype=torch.float64).view(1, 2, 1)
        self.radrow = torch.tensor(T.radial_rows(lay))
        self.mprimary = self.general
        z = ctx.z
        self.g = _G(torch.stack([ctx.src, ctx.dst]), self.V)
        self.gz = _G(torch.stack([z[ctx.src], z[ctx.dst]]), model.max_num_elements)
        self.gn = _G(torch.stack([z, z]), model.max_num_elements)
        self.dexp = _lin(ctx.dist[:, None], model.distance_expansion.weight, model.distance_expansion.bias)
        self.training = model.training
        self.batch = torch.arange(B).repeat_interleave(N)
        ta, fa = EQ.grid_mats(lay.lmax, lay.mmax)
        tf, ff = EQ.grid_mats(lay.lmax, lay.lmax)
        nr, nf = lay.n_red, lay.n_full
        ta, fa = ta.reshape(-1, nr), fa.reshape(-1, nr)
        if self.mprimary:
            ta, fa = ta[:, self.perm], fa[:, self.perm]
        self.grid_attn, self.grid_ffn = (ta, fa), (tf.reshape(-1, nf), ff.reshape(-1, nf))
    monkeypatch.setattr(T._Step, "__init__", step_init)


@pytest.mark.parametrize("lmax,mmax", [(6, 2), (4, 3), (2, 1)])
def test_inference_forward_radial_rows_match_oracle(torch_ops, lmax, mmax):
    """Under no_grad the general path applies SO2_Convolution's radial product inside the gathered
    rotation (rotate_gather_radial) through radial_rows' row map; with that map in a torch stand-in the
    composed forward equals the oracle."""
    torch.manual_seed(1)
    cfg = dict(CFG, lmax_list=[lmax], mmax_list=[mmax])
    m = EquiformerV2_nbody(**cfg, alpha_drop=0.0, drop_path_rate=0.0).double().eval()
    m.specialised_ops = False
    B, N = 2, 4
    rng = np.random.default_rng(1)
    loc = torch.tensor(rng.standard_normal((B * N, 3)))
    vel = torch.tensor(rng.standard_normal((B * N, 3))) * 0.3
    mass = torch.tensor(rng.integers(1, 4, B * N).astype(np.float64))
    gauge = torch.tensor(rng.uniform(0, 1, (B * N * (N - 1), 3)))
    with torch.no_grad():
        got = T.train_forward(m, loc, vel, mass, B, N, gauge, 0)
        P = {k: p.detach().clone() for k, p in m.named_parameters()}
        ref = EQ.forward(cfg, P, loc, vel, mass, B, N, gauge)
    torch.testing.assert_close(got, ref, rtol=0, atol=1e-13)


@pytest.mark.parametrize("lmax,mmax,general", [(2, 1, False), (2, 1, True), (6, 2, True), (4, 3, True), (3, 0, True)])
def test_train_forward_composition_matches_oracle(torch_ops, lmax, mmax, general):
    """The composition's host logic (coefficient orders, SO(2) blocks per m, per-degree SO3_LinearV2,
    m = 0 edge-degree slots, grids) at lmax 2 on the specialised and the general operators and at
    lmax 3-6 (the reference default lmax 6 / mmax 2) on the general ones."""
    torch.manual_seed(0)
    cfg = dict(CFG, lmax_list=[lmax], mmax_list=[mmax])
    m = EquiformerV2_nbody(**cfg, alpha_drop=0.0, drop_path_rate=0.0).double()
    m.specialised_ops = not general
    assert m.uses_general_ops() == general
    with torch.no_grad():
        for k, p in m.named_parameters():
            if k.endswith("bias") or "affine" in k or "norm" in k:
                p.add_(0.1 * torch.randn(p.shape, dtype=p.dtype))
    B, N = 3, 5
    rng = np.random.default_rng(0)
    loc = torch.tensor(rng.standard_normal((B * N, 3)))
    vel = torch.tensor(rng.standard_normal((B * N, 3))) * 0.3
    mass = torch.tensor(rng.integers(1, 4, B * N).astype(np.float64))
    gauge = torch.tensor(rng.uniform(0, 1, (B * N * (N - 1), 3)))
    got = T.train_forward(m, loc, vel, mass, B, N, gauge, 0)
    (got ** 2).sum().backward()
    grads = {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}
    P = {k: p.detach().clone().requires_grad_() for k, p in m.named_parameters()}
    ref = EQ.forward(cfg, P, loc, vel, mass, B, N, gauge)
    (ref ** 2).sum().backward()
    torch.testing.assert_close(got.detach(), ref.detach(), rtol=0, atol=1e-13)
    rg = {k: v.grad for k, v in P.items() if v.grad is not None}
    assert set(grads) == set(rg)
    for k in rg:
        torch.testing.assert_close(grads[k], rg[k], rtol=1e-10, atol=1e-12, msg=k)


def test_train_forward_dropout_sites(torch_ops, monkeypatch):
    """Train-mode dropouts of the composition: alpha dropout at each block's own rate and never in the
    force block (equiformer_v2_nbody.py:362 builds it with alpha_drop=0.0), proj_drop after the
    attention and after the FFN of every block (transformer_block.py:690-706), none in eval mode."""
    calls = []
    real = torch.nn.functional.dropout

    def spy(x, p=0.5, training=True, inplace=False):
        calls.append((tuple(x.shape), p, training))
        return real(x, p, training, inplace)
    monkeypatch.setattr(torch.nn.functional, "dropout", spy)
    torch.manual_seed(0)
    m = EquiformerV2_nbody(**CFG, alpha_drop=0.1, drop_path_rate=0.0, proj_drop=0.2).double()
    B, N = 2, 4
    rng = np.random.default_rng(1)
    loc = torch.tensor(rng.standard_normal((B * N, 3)))
    vel = torch.tensor(rng.standard_normal((B * N, 3))) * 0.3
    mass = torch.ones(B * N, dtype=torch.float64)
    gauge = torch.tensor(rng.uniform(0, 1, (B * N * (N - 1), 3)))
    out = T.train_forward(m.train(), loc, vel, mass, B, N, gauge, 0)
    E, V, C, nh = B * N * (N - 1), B * N, CFG["sphere_channels"], CFG["num_heads"]
    per_block = [((E, nh), 0.1, True), ((V, 1, C), 0.2, True), ((V, 1, C), 0.2, True)]
    assert calls == per_block * CFG["num_layers"], calls
    assert torch.isfinite(out).all()
    calls.clear()
    T.train_forward(m.eval(), loc, vel, mass, B, N, gauge, 0)
    assert calls == []
