"""EquiformerV2 training step on the native operators.

The reference trains EquiformerV2_nbody with ``pred = model(data); loss.backward();
optimizer.step()`` (trainer.py:233-358).  Here a grad-mode ``EquiformerV2_nbody.forward``
(equiformer_v2.py) runs :func:`train_forward`: the forward of
models/equiformer_v2/architecture/equiformer_v2_nbody.py:428-575 (any single resolution lmax <= 6,
separable S2 activations, rms_norm_sh) composed of libnbx operators inside ``torch.autograd.Function`` s whose
backward passes call the same library, so ``loss.backward()`` reaches every ``nn.Parameter`` the
reference's forward uses:

* every nn.Linear / SO(2) ``fc`` = ``ponita_train._LinFn`` (nbx_gemm_f32 + nbx_bias_act), every
  SO3_LinearV2 = ``_SO3LinearFn`` (all degrees in one nbx_gemm_f32_grouped launch), every LayerNorm = ``_LayerNormFn``, SiLU / SmoothLeakyReLU = ``_ActFn``;
* SO3_Rotation.rotate / rotate_inv = ``_RotateFn`` (nbx_eqv2_rotate, lmax 2 / mmax 1) or
  ``_RotateGFn`` (nbx_eqv2_rotate_general with the nbx_eqv2_wigner rows, any lmax <= 6); adjoint pairs;
* the separable S2 activation's grid round trip = ``_S2Fn`` (nbx_eqv2_s2_act);
* the attention softmax over edge_index[1] = ``_SoftmaxFn`` (nbx_segment_softmax);
* EquivariantRMSNormArraySphericalHarmonicsV2 = ``_RMSNormFn`` (nbx_eqv2_rms_norm, lmax 2) or
  ``_RMSNormGFn`` (nbx_eqv2_rms_norm_general);
* gathers x[edge_index[0 / 1]], embedding lookups and the aggregation = ``segnn_train._GatherFn`` /
  ``_SegSumFn`` over CSR tables (no atomics).

Edge frames come from ``nbx_eqv2_train_edges`` / ``nbx_eqv2_edges`` (the inference path's frames and
gauge draws).  Without autograd the same composition is the inference forward of the configurations
the fused kernels do not cover (EquiformerV2_nbody.forward / rollout).
Reshapes, concatenations, the SO(2) complex combine, the radial weighting of the messages and the
dropout masks (alpha dropout, GraphDropPath: transformer_block.py:342-343,686-706, drop.py:51-68,
train mode, torch's RNG) are torch glue.  Arithmetic is fp32 (a float64 module is cast for the step).
"""
from __future__ import annotations

import torch

from . import _lib, so3
from .ponita_train import _LayerNormFn, linear
from .segnn_train import Graph, _GatherFn, _SegSumFn, _at, _dp, _st, colsum, gemm_grouped

_f32 = torch.float32
AVG_DEGREE = 23.395238876342773          # equiformer_v2_nbody.py:36


class _ActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, act):
        X = X.contiguous()
        rows, cols = X.shape[0], X.numel() // max(X.shape[0], 1)
        Y = torch.empty_like(X)
        _lib.check(_lib.lib().nbx_bias_act(rows, cols, _dp(X), cols, None, act, _dp(Y), cols, _st(X)), "nbx_bias_act")
        ctx.save_for_backward(X)
        ctx.act = act
        return Y

    @staticmethod
    def backward(ctx, dY):
        (X,) = ctx.saved_tensors
        rows, cols = X.shape[0], X.numel() // max(X.shape[0], 1)
        dY = dY.contiguous()
        dX = torch.empty_like(X)
        _lib.check(_lib.lib().nbx_bias_act_backward(rows, cols, _dp(X), cols, None, ctx.act, _dp(dY), _dp(dX),
                                                    _st(dX)), "nbx_bias_act_backward")
        return dX, None


def act(X, kind):
    return _ActFn.apply(X, kind)


class _RotateFn(torch.autograd.Function):
    """rotate (inverse = 0): [E][9][C] -> [E][7][C]; rotate_inv (inverse = 1): [E][7][C] -> [E][9][C]."""

    @staticmethod
    def forward(ctx, X, D, inverse, rescale):
        E, _, C = X.shape
        X = X.contiguous()
        out = torch.empty(E, 9 if inverse else 7, C, device=X.device, dtype=_f32)
        _lib.check(_lib.lib().nbx_eqv2_rotate(E, C, _dp(D), _dp(X), X.shape[1] * C, _dp(out), inverse, rescale,
                                              _st(X)), "nbx_eqv2_rotate")
        ctx.save_for_backward(D)
        ctx.mode = (inverse, rescale)
        return out

    @staticmethod
    def backward(ctx, dY):
        (D,) = ctx.saved_tensors
        inverse, rescale = ctx.mode
        dY = dY.contiguous()
        E, _, C = dY.shape
        dX = torch.empty(E, 7 if inverse else 9, C, device=dY.device, dtype=_f32)
        _lib.check(_lib.lib().nbx_eqv2_rotate(E, C, _dp(D), _dp(dY), dY.shape[1] * C, _dp(dX), 1 - inverse, rescale,
                                              _st(dY)), "nbx_eqv2_rotate")
        return dX, None, None, None


class _RotateGFn(torch.autograd.Function):
    """General degrees: rotate (inverse = 0) [E][(lmax+1)^2][C] -> [E][R][C], rotate_inv (inverse = 1)
    [E][R][C] -> [E][(lmax+1)^2][C] with the kept Wigner rows D [E][S]; ``order`` (int32 [R] or None):
    the [E][R][C] row of each kept coefficient (the m-primary order of the SO(2) convolutions)."""

    @staticmethod
    def forward(ctx, X, D, lay, inverse, rescale, order=None):
        E, _, C = X.shape
        X = X.contiguous()
        out = torch.empty(E, lay.n_full if inverse else lay.n_red, C, device=X.device, dtype=_f32)
        _lib.check(_lib.lib().nbx_eqv2_rotate_general(E, C, lay.lmax, lay.mmax, _dp(D), _dp(X), X.shape[1] * C,
                                                      _dp(out), inverse, rescale, _dp(order), _st(X)),
                   "nbx_eqv2_rotate_general")
        ctx.save_for_backward(D, order)
        ctx.mode = (lay, inverse, rescale)
        return out

    @staticmethod
    def backward(ctx, dY):
        D, order = ctx.saved_tensors
        lay, inverse, rescale = ctx.mode
        dY = dY.contiguous()
        E, _, C = dY.shape
        dX = torch.empty(E, lay.n_red if inverse else lay.n_full, C, device=dY.device, dtype=_f32)
        _lib.check(_lib.lib().nbx_eqv2_rotate_general(E, C, lay.lmax, lay.mmax, _dp(D), _dp(dY), dY.shape[1] * C,
                                                      _dp(dX), 1 - inverse, rescale, _dp(order), _st(dY)),
                   "nbx_eqv2_rotate_general")
        return dX, None, None, None, None, None


class _S2Fn(torch.autograd.Function):
    """Separable S2 activation's grid part of X [rows][I][H] with T / F [P][I]."""

    @staticmethod
    def forward(ctx, X, T, F):
        X = X.contiguous()
        rows, I, H = X.shape
        out = torch.empty_like(X)
        _lib.check(_lib.lib().nbx_eqv2_s2_act(rows, I, T.shape[0], H, _dp(T), _dp(F), _dp(X), _dp(out), _st(X)),
                   "nbx_eqv2_s2_act")
        ctx.save_for_backward(X, T, F)
        return out

    @staticmethod
    def backward(ctx, dY):
        X, T, F = ctx.saved_tensors
        rows, I, H = X.shape
        dY = dY.contiguous()
        dX = torch.empty_like(X)
        _lib.check(_lib.lib().nbx_eqv2_s2_act_backward(rows, I, T.shape[0], H, _dp(T), _dp(F), _dp(X), _dp(dY),
                                                       _dp(dX), _st(dX)), "nbx_eqv2_s2_act_backward")
        return dX, None, None


class _SoftmaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, g):
        logits = logits.contiguous()
        nh = logits.shape[1]
        alpha = torch.empty_like(logits)
        _lib.check(_lib.lib().nbx_segment_softmax(g.V, nh, _dp(g.dptr), _dp(g.deid), _dp(logits), _dp(alpha),
                                                  _st(logits)), "nbx_segment_softmax")
        ctx.save_for_backward(alpha)
        ctx.g = g
        return alpha

    @staticmethod
    def backward(ctx, dA):
        (alpha,) = ctx.saved_tensors
        g = ctx.g
        dA = dA.contiguous()
        dL = torch.empty_like(alpha)
        _lib.check(_lib.lib().nbx_segment_softmax_backward(g.V, alpha.shape[1], _dp(g.dptr), _dp(g.deid), _dp(alpha),
                                                           _dp(dA), _dp(dL), _st(dA)), "nbx_segment_softmax_backward")
        return dL, None


class _RMSNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, w, b, eps):
        X = X.contiguous()
        V, _, C = X.shape
        Y = torch.empty_like(X)
        save = torch.empty(2, V, device=X.device, dtype=_f32)
        _lib.check(_lib.lib().nbx_eqv2_rms_norm(V, C, _dp(X), _dp(w), _dp(b), float(eps), _dp(Y), _dp(save), _st(X)),
                   "nbx_eqv2_rms_norm")
        ctx.save_for_backward(X, w, save)
        return Y

    @staticmethod
    def backward(ctx, dY):
        X, w, save = ctx.saved_tensors
        V, _, C = X.shape
        dY = dY.contiguous()
        dX = torch.empty_like(X)
        G = torch.empty(V, 4 * C, device=X.device, dtype=_f32)
        _lib.check(_lib.lib().nbx_eqv2_rms_norm_backward(V, C, _dp(X), _dp(w), _dp(save), _dp(dY), _dp(dX), _dp(G),
                                                         _st(dX)), "nbx_eqv2_rms_norm_backward")
        dwb = colsum(G, V, 4 * C, 4 * C, torch.empty(4 * C, device=X.device, dtype=_f32))
        return dX, dwb[:3 * C].view(3, C), dwb[3 * C:], None


class _RMSNormGFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, w, b, eps, lmax):
        X = X.contiguous()
        V, _, C = X.shape
        Y = torch.empty_like(X)
        save = torch.empty(2, V, device=X.device, dtype=_f32)
        _lib.check(_lib.lib().nbx_eqv2_rms_norm_general(V, lmax, C, _dp(X), _dp(w), _dp(b), float(eps), _dp(Y),
                                                        _dp(save), _st(X)), "nbx_eqv2_rms_norm_general")
        ctx.save_for_backward(X, w, save)
        ctx.lmax = lmax
        return Y

    @staticmethod
    def backward(ctx, dY):
        X, w, save = ctx.saved_tensors
        V, _, C = X.shape
        L1 = ctx.lmax + 1
        dY = dY.contiguous()
        dX = torch.empty_like(X)
        G = torch.empty(V, (L1 + 1) * C, device=X.device, dtype=_f32)
        _lib.check(_lib.lib().nbx_eqv2_rms_norm_general_backward(V, ctx.lmax, C, _dp(X), _dp(w), _dp(save), _dp(dY),
                                                                 _dp(dX), _dp(G), _st(dX)),
                   "nbx_eqv2_rms_norm_general_backward")
        dwb = colsum(G, V, (L1 + 1) * C, (L1 + 1) * C, torch.empty((L1 + 1) * C, device=X.device, dtype=_f32))
        return dX, dwb[:L1 * C].view(L1, C), dwb[L1 * C:], None, None


class _SO3LinearFn(torch.autograd.Function):
    """SO3_LinearV2 (so3.py:695-745): Y[v][i] = W[l(i)] X[v][i] (+ b on i = 0) for X [V][(lmax+1)^2][cin],
    W [lmax+1][cout][cin].  The 2l + 1 rows of degree l of every node are one GEMM operand of V (2l + 1)
    rows through nbx_gemm_f32_grouped's two-level rows, so all degrees run in one launch (forward: one
    GEMM per degree; backward: the input and the weight gradient per degree and the bias gradient as
    the row sums of the l = 0 output gradient, up to 8 per launch), with no per-degree slices, copies
    or concatenations, and the weight gradient leaves in W's own layout."""

    @staticmethod
    def forward(ctx, X, W, b, lmax):
        X = X.contiguous()
        V, S, cin = X.shape
        cout = W.shape[1]
        Y = torch.empty(V, S, cout, device=X.device, dtype=_f32)
        # the bias in the l = 0 GEMM's epilogue
        probs = [(_lib.GEMM_TRANS_B, V * (2 * l + 1), cout, cin, _at(X, l * l * cin), cin, _at(W, l * cout * cin), cin,
                  _at(Y, l * l * cout), cout, 0.0, 2 * l + 1, S * cin, 0, S * cout, _dp(b) if l == 0 else None)
                 for l in range(lmax + 1)]
        for i in range(0, len(probs), 8):
            gemm_grouped(probs[i:i + 8], X.device)
        ctx.save_for_backward(X, W)
        ctx.dims = (lmax, b is not None)
        return Y

    @staticmethod
    def backward(ctx, dY):
        X, W = ctx.saved_tensors
        lmax, has_b = ctx.dims
        V, S, cin = X.shape
        cout = W.shape[1]
        dY = dY.contiguous()
        dX = dWb = None
        probs = []
        if ctx.needs_input_grad[0]:
            dX = torch.empty_like(X)
            probs += [(0, V * (2 * l + 1), cin, cout, _at(dY, l * l * cout), cout, _at(W, l * cout * cin), cin,
                       _at(dX, l * l * cin), cin, 0.0, 2 * l + 1, S * cout, 0, S * cin) for l in range(lmax + 1)]
        want_w, want_b = ctx.needs_input_grad[1], has_b and ctx.needs_input_grad[2]
        if want_w or want_b:
            nw = (lmax + 1) * cout * cin
            dWb = torch.empty(nw + cout, device=X.device, dtype=_f32)
            if want_w:
                probs += [(_lib.GEMM_TRANS_A, cout, cin, V * (2 * l + 1), _at(dY, l * l * cout), cout,
                           _at(X, l * l * cin), cin, _at(dWb, l * cout * cin), cin, 0.0, 2 * l + 1, S * cout, S * cin,
                           0) for l in range(lmax + 1)]
            if want_b:          # row sums of dY's l = 0 rows: op(B) is the column of ones alone
                probs.append((_lib.GEMM_TRANS_A | _lib.GEMM_B_ONES, cout, 1, V, _at(dY, 0), cout, _at(X, 0), 0,
                              _at(dWb, nw), 1, 0.0, 1, S * cout, 0, 0))
        for i in range(0, len(probs), 8):
            gemm_grouped(probs[i:i + 8], X.device)
        dW = dWb[:(lmax + 1) * cout * cin].view(lmax + 1, cout, cin) if want_w else None
        db = dWb[(lmax + 1) * cout * cin:] if want_b else None
        return dX, dW, db, None


class _SO2ConvFn(torch.autograd.Function):
    """SO2_Convolution (so2_ops.py:78-156) on m-primary coefficients x [E][R][cin] -> (out [E][R][cout],
    extra [E][n_extra]) in one grouped GEMM launch per direction.  meta = (n0, (n_1 .. n_mmax), n_extra)
    (coefficients of m = 0 and per m > 0 pair); rad [E][(n0 + sum n_m) cin] or None (the radial
    weights, one per (m, coefficient, channel), shared by the +m / -m rows); W0 / b0 = fc_m0; Wm[m - 1] =
    so2_m_conv[m - 1].fc.weight [2 n_m cout][n_m cin] = [Wr; Wi].
    m = 0: [extra | out0] = (x0 rad0) W0^T + b0, written straight into extra and out's m = 0 rows.
    m > 0: the complex pair product out(+m) = x+ Wr^T - x- Wi^T, out(-m) = x- Wr^T + x+ Wi^T is one
    GEMM of [x+ | x-] against [[Wr, -Wi], [Wi, Wr]], written straight into out's rows of the pair.
    Backward: the weight / input gradients of every block in one launch (bias gradients as row sums,
    NBX_GEMM_B_ONES), the radial products by torch elementwise ops into the gradient buffers."""

    @staticmethod
    def forward(ctx, meta, x, rad, W0, b0, *Wm):
        n0, nms, n_extra = meta
        x = x.contiguous()
        E, R, cin = x.shape
        cout = (W0.shape[0] - n_extra) // n0
        dev = x.device
        starts, roffs = [], []
        s_, r_ = n0, n0 * cin
        for nm in nms:
            starts.append(s_)
            roffs.append(r_)
            s_ += 2 * nm
            r_ += nm * cin
        if rad is not None:
            rad = rad.contiguous()
            x0s = x[:, :n0] * rad[:, :n0 * cin].view(E, n0, cin)
            xms = [x[:, st:st + 2 * nm].view(E, 2, nm, cin) * rad[:, ro:ro + nm * cin].view(E, 1, nm, cin)
                   for nm, st, ro in zip(nms, starts, roffs)]
            A0, lda0 = _at(x0s, 0), n0 * cin
            Am = [(_at(t, 0), 2 * nm * cin) for t, nm in zip(xms, nms)]
        else:
            x0s, xms = None, []
            A0, lda0 = _at(x, 0), R * cin
            Am = [(_at(x, st * cin), R * cin) for st in starts]
        Wb = []
        for W, nm in zip(Wm, nms):
            a = nm * cout
            Wr, Wi = W[:a], W[a:]
            Wb.append(torch.cat([torch.cat([Wr, -Wi], 1), torch.cat([Wi, Wr], 1)], 0))
        out = torch.empty(E, R, cout, device=dev, dtype=_f32)
        extra = torch.empty(E, n_extra, device=dev, dtype=_f32)
        K0 = n0 * cin
        probs = []      # fc_m0's bias in the epilogues of its two GEMMs
        if n_extra:
            probs.append((_lib.GEMM_TRANS_B, E, n_extra, K0, A0, lda0, _at(W0, 0), K0, _at(extra, 0), n_extra, 0.0,
                          1, 0, 0, 0, _dp(b0)))
        probs.append((_lib.GEMM_TRANS_B, E, n0 * cout, K0, A0, lda0, _at(W0, n_extra * K0), K0, _at(out, 0), R * cout,
                      0.0, 1, 0, 0, 0, _at(b0, n_extra) if b0 is not None else None))
        for (ap, lda), Wbm, nm, st in zip(Am, Wb, nms, starts):
            probs.append((_lib.GEMM_TRANS_B, E, 2 * nm * cout, 2 * nm * cin, ap, lda, _at(Wbm, 0), 2 * nm * cin,
                          _at(out, st * cout), R * cout, 0.0, 1, 0, 0, 0))
        for i in range(0, len(probs), 8):
            gemm_grouped(probs[i:i + 8], dev)
        ctx.save_for_backward(x, rad, W0, x0s, *xms, *Wb)
        ctx.meta = (n0, nms, n_extra, starts, roffs, b0 is not None, len(xms))
        return out, extra

    @staticmethod
    def backward(ctx, dout, dextra):
        n0, nms, n_extra, starts, roffs, has_b, nx = ctx.meta
        saved = ctx.saved_tensors
        x, rad, W0, x0s = saved[:4]
        xms, Wb = saved[4:4 + nx], saved[4 + nx:]
        E, R, cin = x.shape
        cout = (W0.shape[0] - n_extra) // n0
        dev = x.device
        dout = dout.contiguous()
        K0, M0 = n0 * cin, n_extra + n0 * cout
        # [d extra | d out0] side by side: one operand for the m = 0 weight and input gradients
        if n_extra:
            G0, ldg = torch.cat([dextra.contiguous(), dout[:, :n0].reshape(E, n0 * cout)], 1), M0
        else:
            G0, ldg = dout, R * cout
        if rad is not None:
            A0, lda0 = _at(x0s, 0), K0
            Am = [(_at(t, 0), 2 * nm * cin) for t, nm in zip(xms, nms)]
        else:
            A0, lda0 = _at(x, 0), R * cin
            Am = [(_at(x, st * cin), R * cin) for st in starts]
        need_x = ctx.needs_input_grad[1]
        dx = torch.empty(E, R, cin, device=dev, dtype=_f32) if need_x or rad is not None else None
        dW0b = torch.empty(M0 * (K0 + 1), device=dev, dtype=_f32)
        dWb = [torch.empty(2 * nm * cout, 2 * nm * cin, device=dev, dtype=_f32) for nm in nms]
        # input-side gradients land in scratch when a radial product follows, else straight in dx
        dx0s = torch.empty(E, K0, device=dev, dtype=_f32) if rad is not None else None
        dxms = [torch.empty(E, 2 * nm * cin, device=dev, dtype=_f32) for nm in nms] if rad is not None else []
        probs = [(_lib.GEMM_TRANS_A | _lib.GEMM_B_ONES | _lib.GEMM_ONES_TAIL, M0, K0 + 1, E, _at(G0, 0), ldg, A0, lda0,
                  _at(dW0b, 0), K0, 0.0, 1, 0, 0, 0)]
        if need_x or rad is not None:
            probs.append((0, E, K0, M0, _at(G0, 0), ldg, _at(W0, 0), K0,
                          _at(dx0s, 0) if rad is not None else _at(dx, 0), K0 if rad is not None else R * cin, 0.0,
                          1, 0, 0, 0))
        for i, ((ap, lda), Wbm, nm, st) in enumerate(zip(Am, Wb, nms, starts)):
            n2o, n2i = 2 * nm * cout, 2 * nm * cin
            probs.append((_lib.GEMM_TRANS_A, n2o, n2i, E, _at(dout, st * cout), R * cout, ap, lda, _at(dWb[i], 0), n2i,
                          0.0, 1, 0, 0, 0))
            if need_x or rad is not None:
                probs.append((0, E, n2i, n2o, _at(dout, st * cout), R * cout, _at(Wbm, 0), n2i,
                              _at(dxms[i], 0) if rad is not None else _at(dx, st * cin),
                              n2i if rad is not None else R * cin, 0.0, 1, 0, 0, 0))
        for i in range(0, len(probs), 8):
            gemm_grouped(probs[i:i + 8], dev)
        drad = None
        if rad is not None:
            drad = torch.empty_like(rad)
            torch.mul(dx0s.view(E, n0, cin), rad[:, :K0].view(E, n0, cin), out=dx[:, :n0])
            torch.mul(dx0s.view(E, n0, cin), x[:, :n0], out=drad[:, :K0].view(E, n0, cin))
            for nm, st, ro, g in zip(nms, starts, roffs, dxms):
                g4 = g.view(E, 2, nm, cin)
                torch.mul(g4, rad[:, ro:ro + nm * cin].view(E, 1, nm, cin), out=dx[:, st:st + 2 * nm].view(E, 2, nm, cin))
                torch.sum(g4 * x[:, st:st + 2 * nm].view(E, 2, nm, cin), 1, out=drad[:, ro:ro + nm * cin].view(E, nm, cin))
        dW0 = dW0b[:M0 * K0].view(M0, K0)
        db0 = dW0b[M0 * K0:] if has_b else None
        dWm = []
        for g, nm in zip(dWb, nms):          # [[Wr, -Wi], [Wi, Wr]] -> (dWr; dWi)
            a, b = nm * cout, nm * cin
            d = torch.empty(2 * a, b, device=dev, dtype=_f32)
            torch.add(g[:a, :b], g[a:, b:], out=d[:a])
            torch.sub(g[a:, :b], g[:a, b:], out=d[a:])
            dWm.append(d)
        return (None, dx if need_x else None, drad, dW0, db0, *dWm)


def _f(t):
    return t.to(_f32).contiguous()


def gather(X, idx_graph, which):
    """Rows X[idx] (X [rows][...]) through a CSR of the index (``which``: "s" = the graph's sources,
    "d" = its destinations)."""
    g = idx_graph
    idx = g.src if which == "s" else g.dst
    ptr, eid = (g.sptr, g.seid) if which == "s" else (g.dptr, g.deid)
    shape = X.shape
    out = _GatherFn.apply(X.reshape(shape[0], -1).contiguous(), idx, ptr, eid)
    return out.view(idx.shape[0], *shape[1:])


class _GatherPairFn(torch.autograd.Function):
    """[X[src] | X[dst]] per coefficient: X [V][S][C] -> [E][S][2C] (the attention's
    torch.cat([x[edge_index[0]], x[edge_index[1]]], 2), transformer_block.py:281-289) as two strided
    gathers into the halves of one buffer; backward: two segment sums over the source / destination
    CSRs reading the halves in place, the second accumulating (no concatenation, copy or add)."""

    @staticmethod
    def forward(ctx, X, g):
        X = X.contiguous()
        V, S, C = X.shape
        E = g.src.shape[0]
        out = torch.empty(E, S, 2 * C, device=X.device, dtype=_f32)
        L = _lib.lib()
        for h, idx in enumerate((g.src, g.dst)):
            _lib.check(L.nbx_gather_rows(E, C, _dp(idx), _dp(X), S * C, C, _at(out, h * C), 2 * S * C, 2 * C, S,
                                         _st(X)), "nbx_gather_rows")
        ctx.g = g
        ctx.shape = (V, S, C)
        return out

    @staticmethod
    def backward(ctx, dout):
        g = ctx.g
        V, S, C = ctx.shape
        dout = dout.contiguous()
        dX = torch.empty(V, S, C, device=dout.device, dtype=_f32)
        L = _lib.lib()
        for h, (ptr, eid) in enumerate(((g.sptr, g.seid), (g.dptr, g.deid))):
            _lib.check(L.nbx_segment_sum(V, C, _dp(ptr), _dp(eid), _at(dout, h * C), 2 * S * C, 2 * C, _dp(dX), S * C,
                                         C, S, h, _st(dout)), "nbx_segment_sum")
        return dX, None


def gather_pair(X, g):
    return _GatherPairFn.apply(X, g)


def radial_rows(lay):
    """Radial block row of each m-primary coefficient row (SO2_Convolution, so2_ops.py:118-121): the m = 0
    rows one each, then per m > 0 the +m and the -m rows of its n_m coefficients sharing one row each."""
    rows, r0 = list(range(lay.m_size[0])), lay.m_size[0]
    for mm in range(1, lay.mmax + 1):
        nm = lay.m_size[mm]
        rows += [r0 + i for i in range(nm)] * 2
        r0 += nm
    return rows


def rotate_gather_radial(X, g, D, lay, order, rad, radrow):
    """Inference only (no autograd): _RotateGatherFn's output times SO2_Convolution's radial weights rad
    [E][(n0 + sum n_m) 2C], fused in the rotation's epilogue (nbx_eqv2_rotate_gather with rad): the
    x * rad product of the convolution (so2_ops.py:118-121) never materialises separately."""
    X, rad = X.contiguous(), rad.contiguous()
    V, K, C = X.shape
    E = g.src.shape[0]
    out = torch.empty(E, lay.n_red, 2 * C, device=X.device, dtype=_f32)
    _lib.check(_lib.lib().nbx_eqv2_rotate_gather(E, C, lay.lmax, lay.mmax, _dp(D), _dp(X), K * C, _dp(g.src),
                                                 _dp(g.dst), _dp(out), 0, _dp(order), _dp(rad), rad.shape[1],
                                                 _dp(radrow), _st(X)), "nbx_eqv2_rotate_gather")
    return out


class _RotateGatherFn(torch.autograd.Function):
    """General degrees: rotate(gather_pair(X, g)) in one pass (nbx_eqv2_rotate_gather): X [V][(lmax+1)^2][C]
    -> [E][R][2C], the [E][(lmax+1)^2][2C] gathered message never written.  Backward: the rotation's
    adjoint (nbx_eqv2_rotate_general, inverse = 1) into the gathered layout, then the gather's two
    segment sums (as _GatherPairFn)."""

    @staticmethod
    def forward(ctx, X, g, D, lay, order):
        X = X.contiguous()
        V, K, C = X.shape
        E = g.src.shape[0]
        out = torch.empty(E, lay.n_red, 2 * C, device=X.device, dtype=_f32)
        _lib.check(_lib.lib().nbx_eqv2_rotate_gather(E, C, lay.lmax, lay.mmax, _dp(D), _dp(X), K * C, _dp(g.src),
                                                     _dp(g.dst), _dp(out), 0, _dp(order), None, 0, None, _st(X)),
                   "nbx_eqv2_rotate_gather")
        ctx.save_for_backward(D, order)
        ctx.g, ctx.lay, ctx.shape = g, lay, (V, K, C)
        return out

    @staticmethod
    def backward(ctx, dY):
        D, order = ctx.saved_tensors
        lay, g = ctx.lay, ctx.g
        V, K, C = ctx.shape
        dY = dY.contiguous()
        E = dY.shape[0]
        dG = torch.empty(E, K, 2 * C, device=dY.device, dtype=_f32)
        L = _lib.lib()
        _lib.check(L.nbx_eqv2_rotate_general(E, 2 * C, lay.lmax, lay.mmax, _dp(D), _dp(dY), dY.shape[1] * 2 * C,
                                             _dp(dG), 1, 0, _dp(order), _st(dY)), "nbx_eqv2_rotate_general")
        dX = torch.empty(V, K, C, device=dY.device, dtype=_f32)
        for h, (ptr, eid) in enumerate(((g.sptr, g.seid), (g.dptr, g.deid))):
            _lib.check(L.nbx_segment_sum(V, C, _dp(ptr), _dp(eid), _at(dG, h * C), 2 * K * C, 2 * C, _dp(dX), K * C,
                                         C, K, h, _st(dG)), "nbx_segment_sum")
        return dX, None, None, None, None


class _Step:
    """Per-forward state: the graph, edge frames, distance expansion and dropout settings."""

    def __init__(self, model, pos, vel, charges, B, N, gauge, seed, frame=0):
        dev = pos.device
        self.m, self.B, self.N = model, B, N
        V, E = B * N, B * N * (N - 1)
        self.V, self.E = V, E
        lay = self.lay = model.layout
        self.general = model.uses_general_ops()
        rot = torch.empty(max(E, 1), 32, device=dev, dtype=_f32)
        dist = torch.empty(max(E, 1), device=dev, dtype=_f32)
        zn = torch.empty(V, device=dev, dtype=torch.int32)
        if self.general:
            self.D = torch.empty(max(E, 1), lay.dsel_floats, device=dev, dtype=_f32)
            _lib.check(_lib.lib().nbx_eqv2_edges(B, N, _dp(pos), _dp(charges), _dp(gauge), seed, frame,
                                                 model.max_num_elements, _dp(rot), _dp(dist), _dp(zn), _st(pos)),
                       "nbx_eqv2_edges")
            _lib.check(_lib.lib().nbx_eqv2_wigner(E, lay.lmax, lay.mmax, _dp(rot), 32,
                                                  _dp(model.wigner_table(dev)), _dp(self.D), _st(pos)),
                       "nbx_eqv2_wigner")
        else:
            if frame:
                raise ValueError("frame > 0 needs the general operators")
            self.D = torch.empty(max(E, 1), 7, 9, device=dev, dtype=_f32)
            _lib.check(_lib.lib().nbx_eqv2_train_edges(B, N, _dp(pos), _dp(charges), _dp(gauge), seed,
                                                       model.max_num_elements, _dp(rot), _dp(self.D), _dp(dist),
                                                       _dp(zn), _st(pos)), "nbx_eqv2_train_edges")
        from .graph import fc_edge_index
        # the fully-connected graph's index tables depend on (B, N) only: built once per shape and device
        gcache = model.__dict__.setdefault("_eqv2_fc_graphs", {})
        if (B, N, dev) not in gcache:
            gcache[(B, N, dev)] = Graph(fc_edge_index(B, N, dev), V, dev)
        self.g = gcache[(B, N, dev)]
        zl = zn.long()
        ze = torch.stack([zl[self.g.src.long()], zl[self.g.dst.long()]])
        self.gz = Graph(ze, model.max_num_elements, dev)          # CSRs of the edges' source / target elements
        self.gn = Graph(torch.stack([zl, zl]), model.max_num_elements, dev)   # of the nodes' elements
        self.dexp = linear(dist[:E, None], model.distance_expansion.weight, model.distance_expansion.bias)
        self.training = model.training
        self.batch = torch.arange(B, device=dev).repeat_interleave(N)
        ga, gf = model.SO3_grid[lay.lmax][lay.mmax], model.SO3_grid[lay.lmax][lay.lmax]
        nr, nf = lay.n_red, lay.n_full
        # coefficient index tables, built once per device (no host-to-device copy inside a captured step)
        cache = model.__dict__.setdefault("_eqv2_index_cache", {})
        if dev not in cache:
            cache[dev] = tuple(torch.tensor(v, device=dev, dtype=torch.long) for v in (lay.perm, lay.inv_perm, lay.m0)) \
                + (torch.tensor(lay.inv_perm, device=dev, dtype=torch.int32),
                   torch.tensor([-1.0, 1.0], device=dev, dtype=_f32).view(1, 2, 1))
        self.perm, self.inv_perm, self.m0, self.order, self.sign = cache[dev]
        # the radial block row of each m-primary row (SO2_Convolution: the m = 0 rows, then per m the +m and
        # -m rows of its n_m coefficients sharing one radial row each); rotate_gather_radial
        rcache = model.__dict__.setdefault("_eqv2_radrow_cache", {})
        if dev not in rcache:
            rcache[dev] = torch.tensor(radial_rows(lay), device=dev, dtype=torch.int32)
        self.radrow = rcache[dev]
        # general operators: edge irreps stay in the m-primary order of the SO(2) convolutions end to end
        # (the rotation writes / reads rows through `order`, the attention grid's columns are permuted
        # once), so no feature permutation runs per convolution; the lmax-2 operators work l-primary
        self.mprimary = self.general
        ta, fa = ga.to_grid_mat.reshape(-1, nr), ga.from_grid_mat.reshape(-1, nr)
        if self.mprimary:
            ta, fa = ta[:, self.perm.to(ta.device)], fa[:, self.perm.to(fa.device)]
        self.grid_attn = (_f(ta), _f(fa))
        self.grid_ffn = (_f(gf.to_grid_mat.reshape(-1, nf)), _f(gf.from_grid_mat.reshape(-1, nf)))

    def rotate(self, x):
        """SO3_Rotation.rotate (so3.py:485-505): [E][(lmax+1)^2][C] -> the kept rows [E][R][C]."""
        if self.general:
            return _RotateGFn.apply(x, self.D, self.lay, 0, 0, self.order)
        return _RotateFn.apply(x, self.D, 0, 0)

    def rotate_inv(self, y):
        """SO3_Rotation.rotate_inv with get_rotate_inv_rescale (so3.py:507-531)."""
        if self.general:
            return _RotateGFn.apply(y, self.D, self.lay, 1, 1, self.order)
        return _RotateFn.apply(y, self.D, 1, 1)

    # ---------------------------------------------------------------- building blocks
    def x_edge(self, mod):
        s = gather(_f(mod.source_embedding.weight), self.gz, "s")
        t = gather(_f(mod.target_embedding.weight), self.gz, "d")
        return torch.cat([self.dexp, s, t], 1)

    @staticmethod
    def rad_func(rad, x):
        """RadialFunction: Linear, LayerNorm, SiLU, Linear, LayerNorm, SiLU, Linear."""
        net = rad.net
        h = linear(x, net[0].weight, net[0].bias)
        h = act(_LayerNormFn.apply(h, _f(net[1].weight), _f(net[1].bias), net[1].eps), _lib.ACT_SILU)
        h = linear(h, net[3].weight, net[3].bias)
        h = act(_LayerNormFn.apply(h, _f(net[4].weight), _f(net[4].bias), net[4].eps), _lib.ACT_SILU)
        return linear(h, net[6].weight, net[6].bias)

    def so2_conv(self, conv, x, x_edge, cout, n_extra=0):
        """SO2_Convolution (so2_ops.py:78-156) of x [E][R][cin] (kept coefficients) -> ([E][R][cout], extra):
        m-primary order (CoefficientMappingModule), the m = 0 block through fc_m0, every m > 0 pair
        (+m, -m) through its SO2_m_Convolution as a complex product (_SO2ConvFn)."""
        lay = self.lay
        xm = x if self.mprimary else x[:, self.perm]
        rad = self.rad_func(conv.rad_func, x_edge) if x_edge is not None else None
        meta = (lay.m_size[0], tuple(lay.m_size[m] for m in range(1, lay.mmax + 1)), n_extra)
        b0 = _f(conv.fc_m0.bias) if conv.fc_m0.bias is not None else None
        out, extra = _SO2ConvFn.apply(meta, xm, rad, _f(conv.fc_m0.weight), b0,
                                      *[_f(c.fc.weight) for c in conv.so2_m_conv])
        return (out if self.mprimary else out[:, self.inv_perm]), extra

    def so3_linear(self, lin, x):
        """SO3_LinearV2 (so3.py:695-745): per-degree weight, bias on l = 0.  x [V][(lmax+1)^2][cin]."""
        return _SO3LinearFn.apply(x, _f(lin.weight), _f(lin.bias) if lin.bias is not None else None, self.lay.lmax)

    def rms_norm(self, norm, x):
        if self.general:
            return _RMSNormGFn.apply(x, _f(norm.affine_weight), _f(norm.affine_bias), norm.eps, self.lay.lmax)
        return _RMSNormFn.apply(x, _f(norm.affine_weight), _f(norm.affine_bias), norm.eps)

    def drop_path(self, x):
        """GraphDropPath (drop.py:51-68): one Bernoulli keep / (1 - p) per system, train mode."""
        p = self.m.drop_path_rate
        if not self.training or p == 0.0:
            return x
        keep = torch.empty(self.B, 1, 1, device=x.device, dtype=x.dtype).bernoulli_(1.0 - p) / (1.0 - p)
        return x * keep[self.batch]

    def proj_drop(self, x):
        """EquivariantDropoutArraySphericalHarmonics(drop_graph=False) (drop.py:121-146), applied to the
        attention and FFN outputs (transformer_block.py:690-706): one keep / (1 - p) per (node, channel),
        shared by all coefficients, train mode."""
        p = self.m.proj_drop
        if not self.training or p == 0.0:
            return x
        mask = torch.nn.functional.dropout(x.new_ones(x.shape[0], 1, x.shape[2]), p, True)
        return x * mask

    # ---------------------------------------------------------------- layers
    def attention(self, A, x, cout):
        """SO2EquivariantGraphAttention (transformer_block.py:226-370) of x [V][9][C] -> [V][9][cout]."""
        m, g, E, V = self.m, self.g, self.E, self.V
        nh, na, nv, H = m.num_heads, m.attn_alpha_channels, m.attn_value_channels, m.attn_hidden_channels
        x_edge = self.x_edge(A)
        if self.general and not torch.is_grad_enabled():   # inference: radial product in the rotation
            rad = self.rad_func(A.so2_conv_1.rad_func, x_edge)
            msg = rotate_gather_radial(x, g, self.D, self.lay, self.order, rad, self.radrow)
            msg, extra = self.so2_conv(A.so2_conv_1, msg, None, H, n_extra=nh * na + H)
        else:
            msg = _RotateGatherFn.apply(x, g, self.D, self.lay, self.order) if self.general \
                else self.rotate(gather_pair(x, g))
            msg, extra = self.so2_conv(A.so2_conv_1, msg, x_edge, H, n_extra=nh * na + H)
        a_in, gating = torch.split(extra, [nh * na, H], dim=1)
        s2 = torch.split(_S2Fn.apply(msg, *self.grid_attn), [1, msg.shape[1] - 1], dim=1)[1]
        msg = torch.cat([act(gating.contiguous(), _lib.ACT_SILU)[:, None], s2], 1)
        msg, _ = self.so2_conv(A.so2_conv_2, msg, None, nh * nv)
        a = _LayerNormFn.apply(a_in.reshape(E * nh, na).contiguous(), _f(A.alpha_norm.weight), _f(A.alpha_norm.bias),
                               A.alpha_norm.eps)
        a = act(a, _lib.ACT_SLRELU).view(E, nh, na)
        logit = (a * _f(A.alpha_dot)).sum(-1)
        alpha = _SoftmaxFn.apply(logit, g)
        if self.training and A.alpha_drop > 0.0:   # the module's own rate: the force block's is 0
            alpha = torch.nn.functional.dropout(alpha, A.alpha_drop, True)    # (equiformer_v2_nbody.py:362)
        nr, nf = self.lay.n_red, self.lay.n_full
        msg = (msg.view(E, nr, nh, nv) * alpha[:, None, :, None]).reshape(E, nr, nh * nv)
        rot = self.rotate_inv(msg)
        agg = _SegSumFn.apply(rot.reshape(E, nf * nh * nv), g.dst, g.dptr, g.deid, V).view(V, nf, nh * nv)
        return self.so3_linear(A.proj, agg)

    def ffn(self, F, x):
        """FeedForwardNetwork (transformer_block.py:473-530), separable S2 activation on SO3_Grid(lmax, lmax)."""
        V, S, C = x.shape
        # the l = 0 columns of each node's row, read in place (leading dimension S C)
        gating = linear(x.reshape(V, S * C), F.gating_linear.weight, F.gating_linear.bias, _lib.ACT_SILU, ldx=S * C)
        h = self.so3_linear(F.so3_linear_1, x)
        s2 = torch.split(_S2Fn.apply(h, *self.grid_ffn), [1, h.shape[1] - 1], dim=1)[1]
        h = torch.cat([gating[:, None], s2], 1)
        return self.so3_linear(F.so3_linear_2, h)

    def edge_degree(self):
        """EdgeDegreeEmbedding (input_block.py:83-138): m = 0 radial coefficients rotated back and
        summed over the incoming edges / AVG_DEGREE."""
        ed, E, V, C = self.m.edge_degree_embedding, self.E, self.V, self.m.sphere_channels
        lay = self.lay
        r = self.rad_func(ed.rad_func, self.x_edge(ed)).view(E, lay.m_size[0], C)
        if self.mprimary:                                                      # m = 0 rows come first
            red = torch.cat([r, r.new_zeros(E, lay.n_red - lay.m_size[0], C)], 1)
        else:
            red = r.new_zeros(E, lay.n_red, C).index_copy(1, self.m0, r)         # the m = 0 slots
        y = self.rotate_inv(red)
        out = _SegSumFn.apply(y.reshape(E, lay.n_full * C), self.g.dst, self.g.dptr, self.g.deid,
                              V).view(V, lay.n_full, C)
        return out / AVG_DEGREE


def train_forward(model, pos, vel, charges, B, N, gauge=None, seed=0, frame=0):
    """equiformer_v2_nbody.py:428-575 with autograd through the native operators.  pos / vel [V, 3],
    charges [V] fp32 on the device; gauge [E, 3] or None (device hash of ``seed`` and ``frame``).
    Returns [V, 6]."""
    m = model
    st = _Step(m, pos, vel, charges, B, N, gauge, seed, frame)
    V, C = st.V, m.sphere_channels
    x0 = gather(_f(m.sphere_embedding.weight), st.gn, "s")                               # [V][C]
    xv = linear(vel, m.velocity_embedding.weight, m.velocity_embedding.bias).view(V, 3, C)
    x = torch.cat([x0[:, None], xv, x0.new_zeros(V, st.lay.n_full - 4, C)], 1) + st.edge_degree()
    for blk in m.blocks:
        y = st.proj_drop(st.drop_path(st.attention(blk.ga, st.rms_norm(blk.norm_1, x), C))) + x
        x = st.proj_drop(st.drop_path(st.ffn(blk.ffn, st.rms_norm(blk.norm_2, y)))) + y
    x = st.rms_norm(m.norm, x)
    pred = st.attention(m.force_block, x, 2)
    return pred[:, 1:4, :2].transpose(1, 2).reshape(V, 6)     # (force l = 1 | velocity l = 1)
