"""torch fp64 autograd restatement of the PONITA fibre-bundle forward — TEST ORACLE ONLY.

The same algorithm as oracle/ponita.py (which follows models/ponita/ponita_nbody.py:82-95,
models/ponita/models/ponita_pg.py:134-192, transforms/position_orientation_graph.py:58-87,
geometry/invariants.py:9-51, nn/embedding.py:4-15, nn/conv.py:65-140, nn/convnext.py:18-32,
utils/to_from_sphere.py:4-14), written with torch ops so that torch autograd gives the parameter
gradients of a training step (trainer.py:233-358, ``loss.backward()``): the reference for the native
PONITA training backward (ponita_train.py, csrc/ponita_train.hip).  Pinned to the numpy oracle's
forward and to the reference's golden vectors in tests/test_oracle_ponita.py, and to finite
differences there.  CPU baseline of ``bench.py --model ponita_train`` (the reference trains PONITA in
float64: config.yaml ``ponita_nbody.double_precision: True``).
"""
from __future__ import annotations

import math

import torch


def gelu(x):
    return 0.5 * x * (1.0 + torch.erf(x / math.sqrt(2.0)))


def poly_features(x, degree=3):
    """nn/embedding.py:4-15: [x, x (x) x, (x (x) x) (x) x, ...] with the previous factor major."""
    feats = [x]
    for _ in range(1, degree):
        prev = feats[-1]
        feats.append((prev[..., :, None] * x[..., None, :]).reshape(x.shape[:-1] + (-1,)))
    return torch.cat(feats, -1)


def lin(p, key, x, bias=True):
    y = x @ p[key + ".weight"].T
    if bias and (key + ".bias") in p:
        y = y + p[key + ".bias"]
    return y


def layer_norm(x, w, b, eps=1e-5):
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * w + b


def invariants(ori_grid, rel_pos):
    """geometry/invariants.py:9-51 -> attr [E, O, 2], fiber_attr [O, O, 1]."""
    r = rel_pos[:, None, :]
    oa = ori_grid[None, :, :]
    ob = ori_grid[:, None, :]
    inv1 = (r * oa).sum(-1, keepdim=True)
    inv2 = torch.sqrt(((r - inv1 * oa) ** 2).sum(-1, keepdim=True))
    inv3 = (oa * ob).sum(-1, keepdim=True)
    return torch.cat([inv1, inv2], -1), inv3


def forward(p, x, vec, edge_index, rel_pos, ori_grid, num_layers, degree=3, multiple_readouts=True,
            out_scalar=0, out_vec=2):
    """x [V, Cs] scalars (mass), vec [V, Cv, 3]; ``p``: {state_dict key: tensor}; returns [V, out_vec*3]."""
    src, dst = edge_index[0], edge_index[1]
    V = x.shape[0]
    O = ori_grid.shape[0]
    xs = x[:, None, :].expand(V, O, x.shape[1])
    xv = torch.einsum("bcd,nd->bnc", vec, ori_grid)
    f = torch.cat([xs, xv], -1)
    attr, fiber_attr = invariants(ori_grid, rel_pos)
    kb = gelu(lin(p, "model.basis_fn.3", gelu(lin(p, "model.basis_fn.1", poly_features(attr, degree)))))
    fkb = gelu(lin(p, "model.fiber_basis_fn.3", gelu(lin(p, "model.fiber_basis_fn.1",
                                                             poly_features(fiber_attr, degree)))))
    h = lin(p, "model.x_embedder", f, bias=False)
    readouts = []
    for i in range(num_layers):
        pre = f"model.interaction_layers.{i}."
        inp = h
        k = lin(p, pre + "conv.kernel", kb, bias=False)                        # [E, O, C]
        x1 = torch.zeros_like(h).index_add(0, dst, k * h[src])                # aggr add at edge_index[1]
        fk = lin(p, pre + "conv.fiber_kernel", fkb, bias=False)                # [O, O, C]
        y = torch.einsum("boc,opc->bpc", x1, fk) / fk.shape[-2] + p[pre + "conv.bias"]
        y = layer_norm(y, p[pre + "norm.weight"], p[pre + "norm.bias"])
        y = lin(p, pre + "linear_2", gelu(lin(p, pre + "linear_1", y)))
        if (pre + "layer_scale") in p:
            y = p[pre + "layer_scale"] * y
        h = y + inp
        if multiple_readouts or i == num_layers - 1:
            readouts.append(lin(p, f"model.read_out_layers.{i}", h))
    readout = sum(readouts) / len(readouts)
    rv = readout[..., out_scalar:out_scalar + out_vec]
    vecs = torch.einsum("bnc,nd->bcd", rv, ori_grid) / O
    return vecs.reshape(V, -1)


def loss_and_grads(params, ori_grid, pos, vel, mass, edge_index, target, num_layers, multiple_readouts=True):
    """MSE loss of the prediction (trainer.py:233-309, nbody TargetCommonLoss default) and the
    gradient of every learnable parameter, fp64.  ``params``: {state_dict key: ndarray}."""
    import numpy as np
    learn = lambda k: not (k.endswith("callibrated") or k.endswith("ori_grid"))
    P = {k: torch.tensor(np.asarray(v), dtype=torch.float64, requires_grad=learn(k)) for k, v in params.items()}
    t = lambda a: torch.as_tensor(np.asarray(a), dtype=torch.float64)
    pos, vel, mass = t(pos), t(vel), t(mass)
    ei = torch.as_tensor(np.asarray(edge_index), dtype=torch.int64)
    out = forward(P, mass.reshape(-1, 1), vel.reshape(-1, 1, 3), ei, pos[ei[0]] - pos[ei[1]], t(ori_grid),
                  num_layers, multiple_readouts=multiple_readouts)
    loss = torch.nn.functional.mse_loss(out, t(target))
    loss.backward()
    grads = {k: v.grad.numpy() for k, v in P.items() if v.grad is not None}
    return float(loss.detach()), out.detach().numpy(), grads


__all__ = ["forward", "loss_and_grads", "gelu", "poly_features", "invariants"]
