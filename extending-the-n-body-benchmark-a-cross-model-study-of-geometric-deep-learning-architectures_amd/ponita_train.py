"""PONITA training step on the native operators.

The reference trains PONITA_NBODY with ``pred = model(graph); loss.backward(); optimizer.step()``
(trainer.py:233-358).  Here a grad-mode ``PONITA_NBODY.forward`` (ponita.py) runs
:func:`train_forward`: the forward of models/ponita/models/ponita_pg.py:134-192 composed of libnbx
operators (include/nbx.h "PONITA training step", csrc/ponita_train.hip, and the fp32 MFMA GEMM /
column sums of csrc/segnn_train.hip) inside ``torch.autograd.Function`` s whose backward passes call
the same library, so ``loss.backward()`` lands on every ``nn.Parameter`` of the reference's module
tree:

* every nn.Linear (+ bias, + GELU) = ``_LinFn``: GEMM, then bias + activation; backward:
  activation backward, a column sum (bias), two GEMMs (input and weight gradients);
* FiberBundleConv (nn/conv.py:103-133): the spatial message over the destination CSR (``_MessageFn``;
  backward over the source CSR, no atomics) and the depth-wise fibre convolution + bias
  (``_FiberFn``);
* LayerNorm (``_LayerNormFn``).

Invariants / polynomial features / the lifted input are data (no gradient), computed once per step
by ``nbx_ponita_train_featurize``; the two basis MLPs run once per step and their outputs are shared
by every layer (autograd sums the per-layer gradients).  The read-out mean and ``sphere_to_vec``
(utils/to_from_sphere.py:10-14, an [O] x [O, 3] contraction of two channels) are torch glue.
Arithmetic is fp32 (a float64 module is cast for the step, like its fp32 inference path).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .segnn_train import Graph, colsum, gemm, gemm_batched, gemm_grouped, _at, _dp, _st, _ws

_f32 = torch.float32


class _LinFn(torch.autograd.Function):
    """Y = act(X W^T + b): X [rows][K] (ld = ldx), W [N][K] (nn.Linear layout), b [N] or None.  The bias
    is added in the GEMM's epilogue (nbx_gemm_f32_grouped), so Z = X W^T + b leaves the GEMM and only an
    activation takes a second launch."""

    @staticmethod
    def forward(ctx, X, W, b, act, ldx):
        L = _lib.lib()
        rows = X.shape[0]
        N, K = W.shape
        Z = torch.empty(rows, N, device=X.device, dtype=_f32)
        if rows and N:
            gemm_grouped([(_lib.GEMM_TRANS_B, rows, N, K, _at(X, 0), ldx, _at(W, 0), K, _at(Z, 0), N, 0.0, 1, 0, 0, 0,
                           _dp(b))], X.device)
        if act == _lib.ACT_NONE:
            Y = Z
        else:
            Y = torch.empty_like(Z)
            _lib.check(L.nbx_bias_act(rows, N, _dp(Z), N, None, act, _dp(Y), N, _st(Z)), "nbx_bias_act")
        ctx.save_for_backward(X, W, b, Z if act != _lib.ACT_NONE else None)
        ctx.dims = (rows, N, K, act, ldx)
        return Y

    @staticmethod
    def backward(ctx, dY):
        L = _lib.lib()
        X, W, b, Z = ctx.saved_tensors
        rows, N, K, act, ldx = ctx.dims
        dev = dY.device
        dY = dY.contiguous()
        if act == _lib.ACT_NONE:
            dZ = dY
        else:
            dZ = torch.empty(rows, N, device=dev, dtype=_f32)
            _lib.check(L.nbx_bias_act_backward(rows, N, _dp(Z), N, None, act, _dp(dY), _dp(dZ), _st(dZ)),
                       "nbx_bias_act_backward")
        db = dW = dX = None
        want_b = b is not None and ctx.needs_input_grad[2]
        # the weight and the input gradient GEMMs in one launch (nbx_gemm_f32_batched); the bias gradient
        # (column sums of dZ) is the last column of the weight gradient against X extended by ones, stored
        # after it (NBX_GEMM_ONES_TAIL): both contiguous, so autograd adopts them without a copy
        probs = []
        if ctx.needs_input_grad[1] or want_b:
            dWe = torch.empty(N * (K + 1), device=dev, dtype=_f32)
            probs.append((_lib.GEMM_TRANS_A | _lib.GEMM_B_ONES | _lib.GEMM_ONES_TAIL, N, K + 1, rows, dZ, N, X, ldx,
                          dWe, K, 0.0))
            dW = dWe[:N * K].view(N, K) if ctx.needs_input_grad[1] else None
            if want_b:
                db = dWe[N * K:]
        if ctx.needs_input_grad[0]:
            dX = torch.zeros(rows, ldx, device=dev, dtype=_f32) if ldx != K else torch.empty(rows, K, device=dev,
                                                                                              dtype=_f32)
            probs.append((0, rows, K, N, dZ, N, W, K, dX, ldx, 0.0))
        gemm_batched(probs)
        return dX, dW, db, None, None


def linear(X, W, b=None, act=_lib.ACT_NONE, ldx=None):
    W = W.to(_f32).contiguous()
    b = b.to(_f32).contiguous() if b is not None else None
    return _LinFn.apply(X.contiguous(), W, b, act, int(ldx if ldx is not None else W.shape[1]))


class _MessageFn(torch.autograd.Function):
    """x1[v][o][c] = sum over the edges e into v of k[e][o][c] h[src_e][o][c] (aggr "add" at
    edge_index[1]); K [E*O][C], H [V*O][C]."""

    @staticmethod
    def forward(ctx, K, H, g, O):
        C = H.shape[1]
        X1 = torch.empty_like(H)
        _lib.check(_lib.lib().nbx_po_message(g.V, O, C, _dp(g.dptr), _dp(g.deid), _dp(g.src), _dp(K), _dp(H),
                                             _dp(X1), _st(H)), "nbx_po_message")
        ctx.save_for_backward(K, H)
        ctx.g, ctx.O = g, O
        return X1

    @staticmethod
    def backward(ctx, dX1):
        K, H = ctx.saved_tensors
        g, O = ctx.g, ctx.O
        C = H.shape[1]
        dX1 = dX1.contiguous()
        dK = torch.empty_like(K) if ctx.needs_input_grad[0] else None
        dH = torch.empty_like(H) if ctx.needs_input_grad[1] else None
        _lib.check(_lib.lib().nbx_po_message_backward(g.V, g.E, O, C, _dp(g.src), _dp(g.dst), _dp(g.sptr),
                                                      _dp(g.seid), _dp(K), _dp(H), _dp(dX1), _dp(dK), _dp(dH),
                                                      _st(dX1)), "nbx_po_message_backward")
        return dK, dH, None, None


class _FiberFn(torch.autograd.Function):
    """x2[v][p][c] = (sum_o x1[v][o][c] fk[o][p][c]) / O + bias[c]; X1 [V*O][C], FK [O*O][C]."""

    @staticmethod
    def forward(ctx, X1, FK, bias, O):
        C = X1.shape[1]
        V = X1.shape[0] // O
        X2 = torch.empty_like(X1)
        _lib.check(_lib.lib().nbx_po_fiber_conv(V, O, C, _dp(X1), _dp(FK), _dp(bias), _dp(X2), _st(X1)),
                   "nbx_po_fiber_conv")
        ctx.save_for_backward(X1, FK)
        ctx.O = O
        return X2

    @staticmethod
    def backward(ctx, dX2):
        L = _lib.lib()
        X1, FK = ctx.saved_tensors
        O = ctx.O
        C = X1.shape[1]
        V = X1.shape[0] // O
        dev = X1.device
        dX2 = dX2.contiguous()
        dX1 = torch.empty_like(X1) if ctx.needs_input_grad[0] else None
        dFK = torch.empty_like(FK) if ctx.needs_input_grad[1] else None
        n = _lib.c_sz()
        _lib.check(L.nbx_po_fiber_conv_workspace_bytes(V, O, C, ctypes.byref(n)), "nbx_po_fiber_conv_workspace_bytes")
        ws = _ws(n.value, dev)
        _lib.check(L.nbx_po_fiber_conv_backward(V, O, C, _dp(X1), _dp(FK), _dp(dX2), _dp(dX1), _dp(dFK), _dp(ws),
                                                n.value, _st(dX2)), "nbx_po_fiber_conv_backward")
        db = colsum(dX2, V * O, C, C, torch.empty(C, device=dev, dtype=_f32)) if ctx.needs_input_grad[2] else None
        return dX1, dFK, db, None


class _LayerNormFn(torch.autograd.Function):
    """nn.LayerNorm(C) (eps 1e-5) of X [rows][C]."""

    @staticmethod
    def forward(ctx, X, w, b, eps):
        rows, C = X.shape
        Y = torch.empty_like(X)
        save = torch.empty(2, rows, device=X.device, dtype=_f32)
        _lib.check(_lib.lib().nbx_layernorm_forward(rows, C, _dp(X), _dp(w), _dp(b), float(eps), _dp(Y), _dp(save),
                                                    _st(X)), "nbx_layernorm_forward")
        ctx.save_for_backward(X, w, save)
        return Y

    @staticmethod
    def backward(ctx, dY):
        X, w, save = ctx.saved_tensors
        rows, C = X.shape
        dev = X.device
        dY = dY.contiguous()
        dX = torch.empty_like(X)
        G = torch.empty(rows, 2 * C, device=dev, dtype=_f32)
        _lib.check(_lib.lib().nbx_layernorm_backward(rows, C, _dp(X), _dp(w), _dp(save), _dp(dY), _dp(dX), _dp(G),
                                                     _st(dX)), "nbx_layernorm_backward")
        dwb = colsum(G, rows, 2 * C, 2 * C, torch.empty(2 * C, device=dev, dtype=_f32))
        return dX, dwb[:C], dwb[C:], None


def featurize(pos, vel, mass, ori, g: Graph):
    """Invariants, polynomial features and the lifted input (no gradient): attr [E*O][16],
    fiber [O*O][4], lift [V*O][2]."""
    dev = pos.device
    O = ori.shape[0]
    attr = torch.empty(max(g.E * O, 1), 16, device=dev, dtype=_f32)
    fiber = torch.empty(O * O, 4, device=dev, dtype=_f32)
    lift = torch.empty(g.V * O, 2, device=dev, dtype=_f32)
    _lib.check(_lib.lib().nbx_ponita_train_featurize(g.V, g.E, O, _dp(pos), _dp(vel), _dp(mass), _dp(ori), _dp(g.src),
                                                     _dp(g.dst), _dp(attr), _dp(fiber), _dp(lift), _st(pos)),
               "nbx_ponita_train_featurize")
    return attr[:g.E * O], fiber, lift


def train_forward(module, pos, vel, mass, edge_index):
    """The PONITA_NBODY forward (ponita_nbody.py:82-95, ponita_pg.py:134-192) with autograd through the
    native operators.  pos / vel [V, 3], mass [V] fp32 on the device; edge_index [2, E] (row = source,
    col = target).  Returns pred [V, 6] fp32."""
    m = module.model
    dev = pos.device
    V = pos.shape[0]
    O, C = m.num_ori, m.hidden_dim
    g = Graph(edge_index, V, dev)
    ori = m.ori_grid.to(_f32).contiguous()
    attr, fiber, lift = featurize(pos, vel, mass, ori, g)
    GELU = _lib.ACT_GELU
    b1, b2 = m.basis_fn[1], m.basis_fn[3]
    kb = linear(linear(attr, b1.weight, b1.bias, GELU, ldx=16), b2.weight, b2.bias, GELU)      # [E*O][Bk]
    f1, f2 = m.fiber_basis_fn[1], m.fiber_basis_fn[3]
    fkb = linear(linear(fiber, f1.weight, f1.bias, GELU, ldx=4), f2.weight, f2.bias, GELU)     # [O*O][Bk]
    h = linear(lift, m.x_embedder.weight)                                                       # [V*O][C]
    readouts = []
    for layer, ro in zip(m.interaction_layers, m.read_out_layers):
        conv = layer.conv
        k = linear(kb, conv.kernel.weight)                                                       # [E*O][C]
        x1 = _MessageFn.apply(k, h, g, O)
        fk = linear(fkb, conv.fiber_kernel.weight)                                               # [O*O][C]
        y = _FiberFn.apply(x1, fk.contiguous(), conv.bias.to(_f32).contiguous(), O)
        y = _LayerNormFn.apply(y, layer.norm.weight.to(_f32).contiguous(), layer.norm.bias.to(_f32).contiguous(),
                               layer.norm.eps)
        y = linear(y, layer.linear_1.weight, layer.linear_1.bias, GELU)
        y = linear(y, layer.linear_2.weight, layer.linear_2.bias)
        if layer.layer_scale is not None:
            y = layer.layer_scale.to(_f32) * y
        h = y + h
        if ro is not None:
            readouts.append(linear(h, ro.weight, ro.bias))
    readout = sum(readouts) / len(readouts)
    s0, nv = module.out_channels_scalar, module.out_channels_vec
    rv = readout.view(V, O, -1)[..., s0:s0 + nv]
    vecs = torch.einsum("bnc,nd->bcd", rv, ori) / O                                              # sphere_to_vec
    return vecs.reshape(V, -1)
