"""torch fp64 autograd restatement of the SEGNN forward — TEST ORACLE ONLY.

The same algorithm as oracle/segnn.py + oracle/e3nn_lite.py (which follow models/segnn/segnn.py:150-304,
models/segnn/o3_building_blocks.py:10-278 and e3nn 0.5.1's FullyConnectedTensorProduct / Gate /
BatchNorm / spherical_harmonics), written with torch ops so that torch autograd gives the parameter
gradients a training step (trainer.py:233-358, ``loss.backward()``) needs: the reference for the
native SEGNN training backward (segnn_train.py, csrc/segnn_train.hip).  It is pinned to the numpy
oracle's forward in tests/test_oracle_segnn.py; parity of both vs e3nn itself is UNPINNED (e3nn is
absent from this image).  CPU baseline of ``bench.py --model segnn_train``.
"""
from __future__ import annotations

import math

import torch

from .e3nn_lite import C_SIGMOID, C_SILU, SH_C0, SH_C1, wigner_3j
from .segnn import SEGNNOracle


def fctp(tp, x1, x2, w):
    """e3nn_lite.FullyConnectedTP.__call__ on torch tensors (mode uvw, component normalisation)."""
    Z = x1.shape[0]
    s1, s2, so = tp.irreps_in1.slices(), tp.irreps_in2.slices(), tp.irreps_out.slices()
    parts = [[] for _ in tp.irreps_out]
    off = 0
    for (i1, i2, io, (m1, m2, mo)), c in zip(tp.instructions, tp.coeffs):
        n = m1 * m2 * mo
        W = w[off:off + n].reshape(m1 * m2, mo)
        off += n
        d1, d2, do = tp.irreps_in1[i1][1].dim, tp.irreps_in2[i2][1].dim, tp.irreps_out[io][1].dim
        C = torch.as_tensor(wigner_3j(tp.irreps_in1[i1][1].l, tp.irreps_in2[i2][1].l, tp.irreps_out[io][1].l),
                            dtype=x1.dtype)
        a = x1[:, s1[i1]].reshape(Z, m1, d1)
        b = x2[:, s2[i2]].reshape(Z, m2, d2)
        t = torch.einsum("zui,zvj,ijk->zkuv", a, b, C).reshape(Z, do, m1 * m2)
        y = (t @ W).permute(0, 2, 1).reshape(Z, mo * do)        # [Z, (w, k)]
        parts[io].append(c * y)
    out = [sum(p) if p else x1.new_zeros(Z, so[io].stop - so[io].start) for io, p in enumerate(parts)]
    return torch.cat(out, 1)


def o3tp(mod, p, prefix, x1, x2):
    """O3TensorProduct: FCTP / sqrt_k_correction + biases on the 0e slices."""
    out = fctp(mod.tp, x1, x2, p[prefix + "tp.weight"])
    out = out / torch.as_tensor(mod.sqrt_k_correction, dtype=out.dtype)
    if len(mod.bias_idx):
        b = torch.zeros(out.shape[1], dtype=out.dtype).index_put((torch.as_tensor(mod.bias_idx),),
                                                                  p[prefix + "biases"])
        out = out + b
    return out


def o3tp_gate(mod, p, prefix, x1, x2):
    out = o3tp(mod, p, prefix, x1, x2)
    ns, ng = mod.n_scalars, mod.n_gates
    s = C_SILU * torch.nn.functional.silu(out[:, :ns])
    g = C_SIGMOID * torch.sigmoid(out[:, ns:ns + ng])
    gated = out[:, ns + ng:]
    segs, i, gi = [s], 0, 0
    for m, ir in mod.gated:
        seg = gated[:, i:i + m * ir.dim].reshape(-1, m, ir.dim)
        segs.append((seg * g[:, gi:gi + m, None]).reshape(-1, m * ir.dim))
        i += m * ir.dim
        gi += m
    return torch.cat(segs, 1)


def batch_norm(x, irreps, weight, bias, running_mean, running_var, training, eps=1e-5, momentum=0.1):
    """e3nn_lite.batch_norm on torch tensors; returns (y, new running mean, new running var)."""
    ix = irm = irv = iw = ib = 0
    fields, new_rm, new_rv = [], [], []
    Z = x.shape[0]
    for m, ir in irreps:
        d = ir.dim
        f = x[:, ix:ix + m * d].reshape(Z, m, d)
        ix += m * d
        if ir.is_scalar():
            if training:
                mu = f.mean(dim=(0, 2))
                new_rm.append((1 - momentum) * running_mean[irm:irm + m] + momentum * mu.detach())
            else:
                mu = running_mean[irm:irm + m]
            irm += m
            f = f - mu[None, :, None]
        if training:
            n = (f ** 2).mean(2).mean(0)
            new_rv.append((1 - momentum) * running_var[irv:irv + m] + momentum * n.detach())
        else:
            n = running_var[irv:irv + m]
        irv += m
        f = f * ((n + eps) ** -0.5 * weight[iw:iw + m])[None, :, None]
        iw += m
        if ir.is_scalar():
            f = f + bias[ib:ib + m][None, :, None]
            ib += m
        fields.append(f.reshape(Z, m * d))
    y = torch.cat(fields, 1)
    rm = torch.cat(new_rm) if (training and new_rm) else running_mean
    rv = torch.cat(new_rv) if (training and new_rv) else running_var
    return y, rm, rv


def sh_l1(x):
    n = torch.sqrt((x * x).sum(-1, keepdim=True))
    xh = x / torch.clamp(n, min=1e-12)
    return torch.cat([torch.full_like(x[:, :1], SH_C0), SH_C1 * xh], -1)


def o3_transform(pos, vel, mass, edge_index):
    """O3Transform.__call__ (o3_building_blocks.py:231-278) in torch."""
    src, dst = edge_index
    V = pos.shape[0]
    rel = pos[src] - pos[dst]
    dist = torch.sqrt((rel ** 2).sum(1, keepdim=True))
    ea = sh_l1(rel)
    acc = torch.zeros(V, 4, dtype=pos.dtype).index_add_(0, dst, ea)
    cnt = torch.zeros(V, 1, dtype=pos.dtype).index_add_(0, dst, torch.ones(len(dst), 1, dtype=pos.dtype))
    na = acc / torch.clamp(cnt, min=1.0) + sh_l1(vel)
    x = torch.cat([pos - pos.mean(1, keepdim=True), vel, torch.sqrt((vel ** 2).sum(1, keepdim=True))], 1)
    amf = torch.cat([dist, mass[src] * mass[dst]], -1)
    return x, ea, na, amf


def forward(om: SEGNNOracle, p, pos, vel, mass, edge_index, training=True):
    """SEGNNOracle.forward in torch: ``p`` maps state_dict keys to tensors (the learnable ones may
    require grad).  Returns (out [V, 6], {running stat key: new value})."""
    x, ea, na, amf = o3_transform(pos, vel, mass, edge_index)
    na = torch.cat([torch.ones_like(na[:, :1]), na[:, 1:]], 1)          # catch_isolated_nodes
    src, dst = edge_index
    V = x.shape[0]
    stats = {}
    h = o3tp(om.embedding, p, "embedding_layer.", x, na)
    for i in range(om.num_layers):
        pre = f"layers.{i}."
        m = o3tp_gate(om.ml1, p, pre + "message_layer_1.", torch.cat([h[dst], h[src], amf], -1), ea)
        m = o3tp_gate(om.ml2, p, pre + "message_layer_2.", m, ea)
        k = pre + "message_norm."
        m, stats[k + "running_mean"], stats[k + "running_var"] = batch_norm(
            m, om.hidden_irreps, p[k + "weight"], p[k + "bias"], p[k + "running_mean"], p[k + "running_var"], training)
        agg = torch.zeros(V, m.shape[1], dtype=m.dtype).index_add_(0, dst, m)
        u = o3tp_gate(om.ul1, p, pre + "update_layer_1.", torch.cat([h, agg], -1), na)
        u = o3tp(om.ul2, p, pre + "update_layer_2.", u, na)
        h = h + u
        k = pre + "feature_norm."
        h, stats[k + "running_mean"], stats[k + "running_var"] = batch_norm(
            h, om.hidden_irreps, p[k + "weight"], p[k + "bias"], p[k + "running_mean"], p[k + "running_var"], training)
    h = o3tp_gate(om.pre_pool1, p, "pre_pool1.", h, na)
    return o3tp(om.pre_pool2, p, "pre_pool2.", h, na), stats


def loss_and_grads(om, params, pos, vel, mass, edge_index, target, training=True):
    """MSE loss of the prediction (trainer.py:233-309 with the nbody TargetCommonLoss default) and
    the gradients of every learnable parameter, fp64.  ``params``: {state_dict key: ndarray}."""
    import numpy as np
    P = {k: torch.tensor(np.asarray(v), dtype=torch.float64, requires_grad="running" not in k)
         for k, v in params.items()}
    t = lambda a: torch.as_tensor(np.asarray(a), dtype=torch.float64)
    out, stats = forward(om, P, t(pos), t(vel), t(mass), torch.as_tensor(np.asarray(edge_index)), training)
    loss = torch.nn.functional.mse_loss(out, t(target))
    loss.backward()
    grads = {k: v.grad.numpy() for k, v in P.items() if v.grad is not None}
    return float(loss), out.detach().numpy(), grads, {k: v.numpy() for k, v in stats.items()}


__all__ = ["forward", "loss_and_grads", "o3_transform", "math"]
