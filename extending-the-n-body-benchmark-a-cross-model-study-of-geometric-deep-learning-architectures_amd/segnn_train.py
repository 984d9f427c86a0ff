"""SEGNN training step on the native operators.

The reference trains SEGNN with ``pred = model(graph); loss.backward(); optimizer.step()``
(trainer.py:233-358) in train mode (batch-statistic BatchNorm, segnn.py:233-235,257-261).  Here a
grad-mode ``SEGNN.forward`` (segnn.py) runs :func:`train_forward`: the forward of
models/segnn/segnn.py:150-304 composed of the libnbx training operators (include/nbx.h "SEGNN
training step", csrc/segnn_train.hip) inside ``torch.autograd.Function`` s whose backward passes
call the same library, so ``loss.backward()`` lands on every ``nn.Parameter`` of the reference's
module tree (tensor-product weights, biases, BatchNorm weight / bias):

* every O(3) tensor product (o3_building_blocks.py:10-203) = ``_TPFn``: tp_prep, two MFMA GEMMs
  (scalar rows, vector component planes), tp_post (bias, e3nn Gate, residual); backward: tp_post
  backward, four GEMMs (input and weight gradients), a column sum (bias), tp_prep backward;
* e3nn BatchNorm with batch statistics = ``_BNFn`` (fixed-order fp64 reductions, the running
  statistics updated in place like the reference module);
* message passing (x_i = x[dst], x_j = x[src], aggr="add" at edge_index[1]) = ``_GatherFn`` /
  ``_SegSumFn`` over CSR tables of the edges by destination and by source (deterministic).

The weight operands come from the e3nn parameters through one traced gather (``SEGNN.train_operands``:
every operand element is a constant times one weight element, the layout of ``SEGNN.train_matrices``),
whose backward scatters the operand gradients back onto the parameters.
Arithmetic is fp32 (a float64 module is cast for the step, like its fp32 inference path).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib

_f32 = torch.float32


def _dp(t):
    return _lib.dev_ptr(t) if t is not None else None


def _at(t, offset):
    """Device pointer of element `offset` of the contiguous fp32 tensor t (column slices passed to the
    strided operators with their own leading dimension)."""
    return _lib.dev_ptr(t) + 4 * int(offset)


def _st(t):
    return _lib.stream_ptr(t.device)


def _ws(nbytes, device):
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)


# bench.py's roofline: when a list, every GEMM appends (start event, stop event, flops) recorded on
# the launch stream around its launches
gemm_timer = None


def gemm(flags, M, N, K, A, lda, B, ldb, C, ldc, beta=0.0):
    """C = op(A) op(B) (+ C) through nbx_gemm_f32 (include/nbx.h)."""
    L = _lib.lib()
    n = _lib.c_sz()
    _lib.check(L.nbx_gemm_f32_workspace_bytes(M, N, K, ctypes.byref(n)), "nbx_gemm_f32_workspace_bytes")
    ws = _ws(n.value, C.device) if n.value else None
    if gemm_timer is not None:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
    _lib.check(L.nbx_gemm_f32(flags, M, N, K, _dp(A), lda, _dp(B), ldb, _dp(C), ldc, float(beta), _dp(ws),
                              n.value, _st(C)), "nbx_gemm_f32")
    if gemm_timer is not None:
        ev[1].record()
        gemm_timer.append((ev[0], ev[1], 2.0 * M * N * K))
    return C


def gemm_batched(problems):
    """Up to 4 independent GEMMs ``(flags, M, N, K, A, lda, B, ldb, C, ldc, beta)`` in one launch
    (nbx_gemm_f32_batched: each result bit-identical to nbx_gemm_f32).  Returns the C tensors."""
    problems = [p for p in problems if p[1] > 0 and p[2] > 0]
    if not problems:
        return []
    L = _lib.lib()
    n = len(problems)
    flags = (ctypes.c_int32 * n)(*[int(p[0]) for p in problems])
    dims = (ctypes.c_int64 * (6 * n))(*[int(v) for p in problems for v in (p[1], p[2], p[3], p[5], p[7], p[9])])
    ptr = lambda i: (ctypes.c_void_p * n)(*[_dp(p[i]) for p in problems])
    beta = (ctypes.c_float * n)(*[float(p[10]) for p in problems])
    nb = _lib.c_sz()
    _lib.check(L.nbx_gemm_f32_batched_workspace_bytes(n, dims, ctypes.byref(nb)), "nbx_gemm_f32_batched_workspace_bytes")
    C = problems[0][8]
    ws = _ws(nb.value, C.device) if nb.value else None
    if gemm_timer is not None:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
    _lib.check(L.nbx_gemm_f32_batched(n, flags, dims, ptr(4), ptr(6), ptr(8), beta, _dp(ws), nb.value, _st(C)),
               "nbx_gemm_f32_batched")
    if gemm_timer is not None:
        ev[1].record()
        gemm_timer.append((ev[0], ev[1], sum(2.0 * p[1] * p[2] * p[3] for p in problems)))
    return [p[8] for p in problems]


def gemm_grouped(problems, device):
    """Up to 8 GEMMs with two-level rows in one launch (nbx_gemm_f32_grouped): problems
    ``(flags, M, N, K, A, lda, B, ldb, C, ldc, beta, rdiv, oa, ob, oc[, bias])`` where A / B / C / bias
    are device pointers (ints, e.g. ``_at(t, offset)``; bias None = none); outer strides 0 = plain rows."""
    problems = [p for p in problems if p[1] > 0 and p[2] > 0]
    if not problems:
        return
    L = _lib.lib()
    n = len(problems)
    flags = (ctypes.c_int32 * n)(*[int(p[0]) for p in problems])
    dims = (ctypes.c_int64 * (10 * n))(*[int(v) for p in problems
                                         for v in (p[1], p[2], p[3], p[5], p[7], p[9], p[11], p[12], p[13], p[14])])
    ptr = lambda i: (ctypes.c_void_p * n)(*[int(p[i]) for p in problems])
    beta = (ctypes.c_float * n)(*[float(p[10]) for p in problems])
    bias = (ctypes.c_void_p * n)(*[(int(p[15]) if len(p) > 15 and p[15] else None) for p in problems])
    nb = _lib.c_sz()
    _lib.check(L.nbx_gemm_f32_grouped_workspace_bytes(n, dims, ctypes.byref(nb)), "nbx_gemm_f32_grouped_workspace_bytes")
    ws = _ws(nb.value, device) if nb.value else None
    if gemm_timer is not None:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
    _lib.check(L.nbx_gemm_f32_grouped(n, flags, dims, ptr(4), ptr(6), ptr(8), beta, bias, _dp(ws), nb.value,
                                      _lib.stream_ptr(device)), "nbx_gemm_f32_grouped")
    if gemm_timer is not None:
        ev[1].record()
        gemm_timer.append((ev[0], ev[1], sum(2.0 * p[1] * p[2] * p[3] for p in problems)))


def colsum(X, rows, cols, ld, out, accumulate=False):
    L = _lib.lib()
    n = _lib.c_sz()
    _lib.check(L.nbx_colsum_workspace_bytes(rows, cols, ctypes.byref(n)), "nbx_colsum_workspace_bytes")
    ws = _ws(n.value, out.device)
    _lib.check(L.nbx_colsum(rows, cols, _dp(X), ld, _dp(out), int(accumulate), _dp(ws), n.value, _st(out)),
               "nbx_colsum")
    return out


class _TPFn(torch.autograd.Function):
    """One O(3) tensor product in the canonical form of include/nbx.h ("SEGNN training step").
    XS [rows][Ks], XV [3][rows][Kv] (or None), Y3 [rows][3]; Ws [NSc + Nt][Ks + Kv], Wv [Nt][Kv];
    bias [NSc] or None; residuals RS [rows][Ms] / RV [3][rows][Nt] or None.  Returns (OS, OV)."""

    @staticmethod
    def forward(ctx, XS, XV, Y3, Ws, Wv, bias, RS, RV, Ms, Nt, gate):
        L = _lib.lib()
        dev = XS.device
        rows, Ks = XS.shape
        Kv = XV.shape[2] if XV is not None else 0
        nsc = Ms + (Nt if gate else 0)
        S = torch.empty(rows, Ks + Kv, device=dev, dtype=_f32)
        _lib.check(L.nbx_tp_prep(rows, Ks, Kv, _dp(XS), Ks, _dp(XV), _dp(Y3), _dp(S), _st(S)), "nbx_tp_prep")
        Zs = torch.empty(rows, nsc + Nt, device=dev, dtype=_f32)
        Zv = torch.empty(3, rows, Nt, device=dev, dtype=_f32)
        # the scalar-row and the vector-plane GEMM in one launch
        gemm_batched([(_lib.GEMM_TRANS_B, rows, nsc + Nt, Ks + Kv, S, Ks + Kv, Ws, Ks + Kv, Zs, nsc + Nt, 0.0)] +
                     ([(_lib.GEMM_TRANS_B, 3 * rows, Nt, Kv, XV, Kv, Wv, Kv, Zv, Nt, 0.0)] if Kv else []))
        if not Kv:
            Zv.zero_()
        OS = torch.empty(rows, Ms, device=dev, dtype=_f32)
        OV = torch.empty(3, rows, Nt, device=dev, dtype=_f32)
        _lib.check(L.nbx_tp_post(rows, Ms, Nt, int(gate), _dp(Zs), _dp(Zv), _dp(Y3), _dp(bias), _dp(RS), _dp(RV),
                                 _dp(OS), _dp(OV), _st(OS)), "nbx_tp_post")
        ctx.save_for_backward(S, XV, Y3, Ws, Wv, bias, Zs, Zv)
        ctx.dims = (rows, Ks, Kv, Ms, Nt, nsc, int(gate), RS is not None, RV is not None)
        return OS, OV

    @staticmethod
    def backward(ctx, dOS, dOV):
        L = _lib.lib()
        S, XV, Y3, Ws, Wv, bias, Zs, Zv = ctx.saved_tensors
        rows, Ks, Kv, Ms, Nt, nsc, gate, has_rs, has_rv = ctx.dims
        dev = S.device
        dOS = dOS.contiguous() if dOS is not None else torch.zeros(rows, Ms, device=dev, dtype=_f32)
        dOV = dOV.contiguous() if dOV is not None else torch.zeros(3, rows, Nt, device=dev, dtype=_f32)
        dZs = torch.empty_like(Zs)
        dZv = torch.empty_like(Zv)
        _lib.check(L.nbx_tp_post_backward(rows, Ms, Nt, gate, _dp(Zs), _dp(Zv), _dp(Y3), _dp(bias), _dp(dOS),
                                          _dp(dOV), _dp(dZs), _dp(dZv), _st(dZs)), "nbx_tp_post_backward")
        dbias = None
        want_b = bias is not None and ctx.needs_input_grad[5]
        # the (up to) four backward GEMMs -- weight gradients and input gradients -- in one launch; the
        # bias gradient (column sums of dZs[:, :NSc]) is the last column of the weight-gradient GEMM
        # against S_in extended by a column of ones (NBX_GEMM_B_ONES), stored after the weight gradient
        # (NBX_GEMM_ONES_TAIL) so that both leave contiguous (autograd adopts them without a copy)
        probs = []
        dWs = dWv = dS = None
        if ctx.needs_input_grad[3] or want_b:
            W1, nw = Ks + Kv + 1, (nsc + Nt) * (Ks + Kv)
            dWe = torch.empty((nsc + Nt) * W1, device=dev, dtype=_f32)
            probs.append((_lib.GEMM_TRANS_A | _lib.GEMM_B_ONES | _lib.GEMM_ONES_TAIL, nsc + Nt, W1, rows, dZs, nsc + Nt,
                          S, Ks + Kv, dWe, Ks + Kv, 0.0))
            dWs = dWe[:nw].view(nsc + Nt, Ks + Kv) if ctx.needs_input_grad[3] else None
            if want_b:
                dbias = dWe[nw:nw + nsc]
        if Kv and ctx.needs_input_grad[4]:
            dWv = torch.empty(Nt, Kv, device=dev, dtype=_f32)
            probs.append((_lib.GEMM_TRANS_A, Nt, Kv, 3 * rows, dZv, Nt, XV, Kv, dWv, Kv, 0.0))
        dXS = dXV = None
        need_x = ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
        if need_x:
            dS = torch.empty(rows, Ks + Kv, device=dev, dtype=_f32)
            probs.append((0, rows, Ks + Kv, nsc + Nt, dZs, nsc + Nt, Ws, Ks + Kv, dS, Ks + Kv, 0.0))
            dXS = torch.empty(rows, Ks, device=dev, dtype=_f32)
            if Kv:
                dXV = torch.empty(3, rows, Kv, device=dev, dtype=_f32)
                probs.append((0, 3 * rows, Kv, Nt, dZv, Nt, Wv, Kv, dXV, Kv, 0.0))
        gemm_batched(probs)
        if need_x:
            _lib.check(L.nbx_tp_prep_backward(rows, Ks, Kv, _dp(dS), _dp(Y3), _dp(dXS), Ks, _dp(dXV), _st(dS)),
                       "nbx_tp_prep_backward")
        return (dXS, dXV, None, dWs, dWv, dbias, dOS if has_rs else None, dOV if has_rv else None, None, None, None)


def tp(XS, XV, Y3, Ws, Wv, bias, Ms, Nt, gate, RS=None, RV=None):
    f = lambda t: t.contiguous() if t is not None else None
    return _TPFn.apply(f(XS), f(XV), f(Y3), f(Ws), f(Wv), f(bias), f(RS), f(RV), Ms, Nt, gate)


class _BNFn(torch.autograd.Function):
    """e3nn BatchNorm with batch statistics of (S [rows][M], V [3][rows][M]); the running statistics
    (fp32 tensors rm [M], rv [2M]) are updated in place."""

    @staticmethod
    def forward(ctx, S, V, weight, bias, rm, rv, eps, momentum):
        L = _lib.lib()
        rows, M = S.shape
        dev = S.device
        n = _lib.c_sz()
        _lib.check(L.nbx_bn_train_workspace_bytes(rows, M, ctypes.byref(n)), "nbx_bn_train_workspace_bytes")
        ws = _ws(n.value, dev)
        save = torch.empty(3, M, device=dev, dtype=_f32)
        OS, OV = torch.empty_like(S), torch.empty_like(V)
        _lib.check(L.nbx_bn_train_forward(rows, M, _dp(S), _dp(V), _dp(weight), _dp(bias), _dp(rm), _dp(rv),
                                          float(eps), float(momentum), _dp(save), _dp(OS), _dp(OV), _dp(ws), n.value,
                                          _st(S)), "nbx_bn_train_forward")
        ctx.save_for_backward(S, V, weight, save)
        ctx.wsb = n.value
        return OS, OV

    @staticmethod
    def backward(ctx, dOS, dOV):
        L = _lib.lib()
        S, V, weight, save = ctx.saved_tensors
        rows, M = S.shape
        dev = S.device
        dOS = dOS.contiguous() if dOS is not None else torch.zeros_like(S)
        dOV = dOV.contiguous() if dOV is not None else torch.zeros_like(V)
        ws = _ws(ctx.wsb, dev)
        dS, dV = torch.empty_like(S), torch.empty_like(V)
        dw = torch.empty(2 * M, device=dev, dtype=_f32)
        db = torch.empty(M, device=dev, dtype=_f32)
        _lib.check(L.nbx_bn_train_backward(rows, M, _dp(S), _dp(V), _dp(weight), _dp(save), _dp(dOS), _dp(dOV),
                                           _dp(dS), _dp(dV), _dp(dw), _dp(db), _dp(ws), ctx.wsb, _st(dS)),
                   "nbx_bn_train_backward")
        return dS, dV, dw, db, None, None, None, None


class _SyncBNFn(torch.autograd.Function):
    """_BNFn with the batch statistics of every rank of ``group`` (sharded train-mode BatchNorm): the
    local fixed-order sums [3M + 1] (with the row count) are all-reduced between nbx_bn_train_sums and
    nbx_bn_train_apply; the backward all-reduces (sum dy, sum dy xhat, sum dy_v . v) the same way, while
    dweight / dbias come from the local sums (the data-parallel gradient all-reduce sums them)."""

    @staticmethod
    def forward(ctx, S, V, weight, bias, rm, rv, eps, momentum, group):
        import torch.distributed as dist
        L = _lib.lib()
        rows, M = S.shape
        dev = S.device
        n = _lib.c_sz()
        _lib.check(L.nbx_bn_train_workspace_bytes(rows, M, ctypes.byref(n)), "nbx_bn_train_workspace_bytes")
        ws = _ws(n.value, dev)
        sums = torch.empty(3 * M + 1, device=dev, dtype=torch.float64)
        _lib.check(L.nbx_bn_train_sums(rows, M, _dp(S), _dp(V), None, None, None, _dp(sums), _dp(ws), n.value, _st(S)),
                   "nbx_bn_train_sums")
        dist.all_reduce(sums, group=group)
        save = torch.empty(3, M, device=dev, dtype=_f32)
        OS, OV = torch.empty_like(S), torch.empty_like(V)
        _lib.check(L.nbx_bn_train_apply(rows, M, _dp(S), _dp(V), _dp(weight), _dp(bias), _dp(sums), _dp(rm), _dp(rv),
                                        float(eps), float(momentum), _dp(save), _dp(OS), _dp(OV), _st(S)),
                   "nbx_bn_train_apply")
        ctx.save_for_backward(S, V, weight, save)
        ctx.wsb, ctx.group = n.value, group
        return OS, OV

    @staticmethod
    def backward(ctx, dOS, dOV):
        import torch.distributed as dist
        L = _lib.lib()
        S, V, weight, save = ctx.saved_tensors
        rows, M = S.shape
        dev = S.device
        dOS = dOS.contiguous() if dOS is not None else torch.zeros_like(S)
        dOV = dOV.contiguous() if dOV is not None else torch.zeros_like(V)
        ws = _ws(ctx.wsb, dev)
        local = torch.empty(3 * M + 1, device=dev, dtype=torch.float64)
        _lib.check(L.nbx_bn_train_sums(rows, M, _dp(S), _dp(V), _dp(dOS), _dp(dOV), _dp(save), _dp(local), _dp(ws),
                                       ctx.wsb, _st(S)), "nbx_bn_train_sums")
        dw = torch.empty(2 * M, device=dev, dtype=_f32)
        db = torch.empty(M, device=dev, dtype=_f32)
        scratch = torch.empty(3 * M, device=dev, dtype=torch.float64)
        _lib.check(L.nbx_bn_train_param_grads(M, _dp(save), _dp(local), _dp(scratch), _dp(dw), _dp(db), _st(S)),
                   "nbx_bn_train_param_grads")
        dist.all_reduce(local, group=ctx.group)
        dS, dV = torch.empty_like(S), torch.empty_like(V)
        _lib.check(L.nbx_bn_train_backward_apply(rows, M, _dp(S), _dp(V), _dp(weight), _dp(save), _dp(local),
                                                 _dp(dOS), _dp(dOV), _dp(dS), _dp(dV), _st(S)),
                   "nbx_bn_train_backward_apply")
        return dS, dV, dw, db, None, None, None, None, None


class Graph:
    """Index tables of one edge list: src / dst int32 [E] and CSRs of the edges by destination and by
    source (ptr [V + 1], eid [E]), built on the device without a host synchronisation."""

    def __init__(self, edge_index, V, device):
        ei = edge_index.to(device=device, dtype=torch.int64)
        self.V, self.E = V, ei.shape[1]
        self.src = ei[0].to(torch.int32).contiguous()
        self.dst = ei[1].to(torch.int32).contiguous()
        nodes = torch.arange(V + 1, device=device, dtype=torch.int64)
        for name, key in (("d", ei[1]), ("s", ei[0])):
            order = torch.argsort(key, stable=True)
            ptr = torch.searchsorted(key[order].contiguous(), nodes).to(torch.int32).contiguous()
            setattr(self, name + "ptr", ptr)
            setattr(self, name + "eid", order.to(torch.int32).contiguous())


class _GatherFn(torch.autograd.Function):
    """out[e] = X[idx[e]] per plane (X [planes][V][C] or [V][C]); backward: segment sum over the
    CSR of idx."""

    @staticmethod
    def forward(ctx, X, idx, ptr, eid):
        planes = X.shape[0] if X.dim() == 3 else 1
        V, C = X.shape[-2], X.shape[-1]
        n = idx.shape[0]
        out = torch.empty(*((planes,) if X.dim() == 3 else ()), n, C, device=X.device, dtype=_f32)
        _lib.check(_lib.lib().nbx_gather_rows(n, C, _dp(idx), _dp(X), C, V * C, _dp(out), C, n * C, planes, _st(X)),
                   "nbx_gather_rows")
        ctx.save_for_backward(ptr, eid)
        ctx.shape = (planes, V, C, n, X.dim())
        return out

    @staticmethod
    def backward(ctx, dout):
        ptr, eid = ctx.saved_tensors
        planes, V, C, n, nd = ctx.shape
        dout = dout.contiguous()
        dX = torch.empty(*((planes,) if nd == 3 else ()), V, C, device=dout.device, dtype=_f32)
        _lib.check(_lib.lib().nbx_segment_sum(V, C, _dp(ptr), _dp(eid), _dp(dout), C, n * C, _dp(dX), C, V * C,
                                              planes, 0, _st(dout)), "nbx_segment_sum")
        return dX, None, None, None


class _SegSumFn(torch.autograd.Function):
    """out[v] = sum of Xe[e] over the edges e with idx[e] = v (CSR ptr / eid of idx); backward: gather."""

    @staticmethod
    def forward(ctx, Xe, idx, ptr, eid, V):
        planes = Xe.shape[0] if Xe.dim() == 3 else 1
        n, C = Xe.shape[-2], Xe.shape[-1]
        out = torch.empty(*((planes,) if Xe.dim() == 3 else ()), V, C, device=Xe.device, dtype=_f32)
        _lib.check(_lib.lib().nbx_segment_sum(V, C, _dp(ptr), _dp(eid), _dp(Xe), C, n * C, _dp(out), C, V * C, planes,
                                              0, _st(Xe)), "nbx_segment_sum")
        ctx.save_for_backward(idx)
        ctx.shape = (planes, V, C, n, Xe.dim())
        return out

    @staticmethod
    def backward(ctx, dout):
        (idx,) = ctx.saved_tensors
        planes, V, C, n, nd = ctx.shape
        dout = dout.contiguous()
        dXe = torch.empty(*((planes,) if nd == 3 else ()), n, C, device=dout.device, dtype=_f32)
        _lib.check(_lib.lib().nbx_gather_rows(n, C, _dp(idx), _dp(dout), C, V * C, _dp(dXe), C, n * C, planes,
                                              _st(dout)), "nbx_gather_rows")
        return dXe, None, None, None, None


class _MsgInputFn(torch.autograd.Function):
    """message_layer_1's per-edge input without concatenation kernels: x[dst] and x[src] gathered
    straight into the column slices of one buffer, plus a constant tail (amf).  hs [V][M] ->
    [E][2M + T] = [hs[dst] | hs[src] | tail]; hv [3][V][M] -> [3][E][2M] = [hv[dst] | hv[src]].
    Backward: two segment sums per input (over the destination / source CSR), the second
    accumulating, read from the column slices of the contiguous output gradient."""

    @staticmethod
    def forward(ctx, hs, hv, tail, g):
        L = _lib.lib()
        V, M = hs.shape
        E, T = g.E, tail.shape[1]
        st = _st(hs)
        S = torch.empty(E, 2 * M + T, device=hs.device, dtype=_f32)
        Vv = torch.empty(3, E, 2 * M, device=hs.device, dtype=_f32)
        for j, idx in enumerate((g.dst, g.src)):
            _lib.check(L.nbx_gather_rows(E, M, _dp(idx), _dp(hs), M, V * M, _at(S, j * M), 2 * M + T, 0, 1, st),
                       "nbx_gather_rows")
            _lib.check(L.nbx_gather_rows(E, M, _dp(idx), _dp(hv), M, V * M, _at(Vv, j * M), 2 * M, E * 2 * M, 3,
                                         st), "nbx_gather_rows")
        S[:, 2 * M:].copy_(tail)
        ctx.g, ctx.dims = g, (V, M, T)
        return S, Vv

    @staticmethod
    def backward(ctx, dS, dVv):
        L = _lib.lib()
        g = ctx.g
        V, M, T = ctx.dims
        E = g.E
        dhs = dhv = None
        if dS is not None:
            dS = dS.contiguous()
            dhs = torch.empty(V, M, device=dS.device, dtype=_f32)
            for j, (ptr, eid) in enumerate(((g.dptr, g.deid), (g.sptr, g.seid))):
                _lib.check(L.nbx_segment_sum(V, M, _dp(ptr), _dp(eid), _at(dS, j * M), 2 * M + T, 0, _dp(dhs), M,
                                             V * M, 1, j, _st(dS)), "nbx_segment_sum")
        if dVv is not None:
            dVv = dVv.contiguous()
            dhv = torch.empty(3, V, M, device=dVv.device, dtype=_f32)
            for j, (ptr, eid) in enumerate(((g.dptr, g.deid), (g.sptr, g.seid))):
                _lib.check(L.nbx_segment_sum(V, M, _dp(ptr), _dp(eid), _at(dVv, j * M), 2 * M, E * 2 * M,
                                             _dp(dhv), M, V * M, 3, j, _st(dVv)), "nbx_segment_sum")
        return dhs, dhv, None, None


def featurize(pos, vel, mass, g: Graph):
    """O3Transform + catch_isolated_nodes (no gradient): na3 [V][3], xs0 [V][1], xv0 [3][V][2],
    rhat [E][3], amf [E][2]."""
    dev = pos.device
    V, E = g.V, g.E
    na3 = torch.empty(V, 3, device=dev, dtype=_f32)
    xs0 = torch.empty(V, 1, device=dev, dtype=_f32)
    xv0 = torch.empty(3, V, 2, device=dev, dtype=_f32)
    rhat = torch.empty(max(E, 1), 3, device=dev, dtype=_f32)
    amf = torch.empty(max(E, 1), 2, device=dev, dtype=_f32)
    _lib.check(_lib.lib().nbx_segnn_train_featurize(V, E, _dp(pos), _dp(vel), _dp(mass), _dp(g.src), _dp(g.dst),
                                                    _dp(g.dptr), _dp(g.deid), _dp(na3), _dp(xs0), _dp(xv0),
                                                    _dp(rhat), _dp(amf), _st(pos)), "nbx_segnn_train_featurize")
    return na3, xs0, xv0, rhat[:E], amf[:E]


def _batch_norm(model, bn, S, V, batch_stats):
    """e3nn BatchNorm of the module ``bn`` (segnn.py BatchNorm): batch statistics through _BNFn (the
    running statistics updated in place; fp32 shadows for a float64 module), else the running
    statistics (an affine map, torch ops)."""
    w, b = bn.weight.to(_f32), bn.bias.to(_f32)
    M = S.shape[1]
    if not batch_stats:
        rm, rv = bn.running_mean.to(_f32), bn.running_var.to(_f32)
        sc = w[:M] / torch.sqrt(rv[:M] + bn.eps)
        return (S - rm) * sc + b, V * (w[M:] / torch.sqrt(rv[M:] + bn.eps))
    rm, rv = bn.running_mean, bn.running_var
    shadow = rm.dtype != _f32 or not rm.is_contiguous()
    if shadow:
        rm, rv = rm.to(_f32).contiguous(), rv.to(_f32).contiguous()
    group = getattr(model, "_bn_group", None)
    if group is not None:    # SyncBN (enable_sync_batchnorm): statistics of the whole sharded batch
        OS, OV = _SyncBNFn.apply(S.contiguous(), V.contiguous(), w.contiguous(), b.contiguous(), rm, rv, bn.eps,
                                 bn.momentum, group)
    else:
        OS, OV = _BNFn.apply(S.contiguous(), V.contiguous(), w.contiguous(), b.contiguous(), rm, rv, bn.eps,
                             bn.momentum)
    if shadow:
        with torch.no_grad():
            bn.running_mean.copy_(rm)
            bn.running_var.copy_(rv)
    return OS, OV


def train_forward(model, pos, vel, mass, edge_index):
    """The SEGNN forward of segnn.py:150-189 with autograd through the native operators.
    pos / vel [V, 3], mass [V] fp32 on the device; edge_index [2, E] (row = source, col = target).
    Returns pred [V, 6] fp32."""
    dev = pos.device
    V = pos.shape[0]
    g = Graph(edge_index, V, dev)
    na3, xs0, xv0, rhat, amf = featurize(pos, vel, mass, g)
    W = model.train_operands(dev)
    M = model.mul
    batch_stats = model._bn_batch()
    hs, hv = tp(xs0, xv0, na3, W["emb_s"], W["emb_v"], W["emb_bias"], M, M, 0)
    for li, layer in enumerate(model.layers):
        p = f"layers.{li}."
        # message(x_i = x[dst], x_j = x[src], additional features) -> two gated TPs -> message BatchNorm
        xin, vin = _MsgInputFn.apply(hs.contiguous(), hv.contiguous(), amf, g)   # [x_i | x_j | amf], [v_i | v_j]
        ms, mv = tp(xin, vin, rhat, W[p + "msg1_s"], W[p + "msg1_v"], W[p + "msg1_bias"], M, M, 1)
        ms, mv = tp(ms, mv, rhat, W[p + "msg2_s"], W[p + "msg2_v"], W[p + "msg2_bias"], M, M, 1)
        ms, mv = _batch_norm(model, layer.message_norm, ms, mv, batch_stats)
        # aggr="add" at edge_index[1]
        a_s = _SegSumFn.apply(ms, g.dst, g.dptr, g.deid, V)
        a_v = _SegSumFn.apply(mv, g.dst, g.dptr, g.deid, V)
        # update: cat(x, agg) -> gated TP -> TP, x + update, feature BatchNorm
        us, uv = tp(torch.cat([hs, a_s], 1), torch.cat([hv, a_v], 2), na3, W[p + "upd1_s"], W[p + "upd1_v"],
                    W[p + "upd1_bias"], M, M, 1)
        hs, hv = tp(us, uv, na3, W[p + "upd2_s"], W[p + "upd2_v"], W[p + "upd2_bias"], M, M, 0, RS=hs, RV=hv)
        hs, hv = _batch_norm(model, layer.feature_norm, hs, hv, batch_stats)
    hs, hv = tp(hs, hv, na3, W["pp1_s"], W["pp1_v"], W["pp1_bias"], M, M, 1)
    _, ov = tp(hs, hv, na3, W["pp2_s"], W["pp2_v"], None, 0, 2, 0)
    return ov.permute(1, 2, 0).reshape(V, 6)      # [V][(copy, xyz)]: 2x1o
