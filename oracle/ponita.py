"""numpy restatement of the PONITA fibre-bundle N-body forward — TEST ORACLE ONLY.

Follows:
* PONITA_NBODY.forward                    models/ponita/ponita_nbody.py:82-95
* PonitaFiberBundle.forward               models/ponita/models/ponita_pg.py:134-192
* PositionOrientationGraph (fibre bundle) models/ponita/transforms/position_orientation_graph.py:58-87
* invariant_attr_r3s2_fiber_bundle        models/ponita/geometry/invariants.py:9-51
* PolynomialFeatures                      models/ponita/nn/embedding.py:4-15
* FiberBundleConv (separable, depthwise)  models/ponita/nn/conv.py:65-140
* ConvNext                                models/ponita/nn/convnext.py:4-32
* vec_to_sphere / sphere_to_vec           models/ponita/utils/to_from_sphere.py:4-14
PolynomialCutoff(radius=None) is the identity window (utils/windowing.py:33-34).
Parameters: ``{state_dict key: ndarray}`` with the reference keys (``model.`` prefix).
"""
from __future__ import annotations

import numpy as np
from scipy.special import erf


def gelu(x):
    return 0.5 * x * (1.0 + erf(x / np.sqrt(2.0)))


def poly_features(x, degree=3):
    feats = [x]
    for _ in range(1, degree):
        prev = feats[-1]
        feats.append((prev[..., :, None] * x[..., None, :]).reshape(x.shape[:-1] + (-1,)))
    return np.concatenate(feats, -1)


def lin(p, key, x, bias=True):
    y = x @ p[key + ".weight"].T
    if bias and (key + ".bias") in p:
        y = y + p[key + ".bias"]
    return y


def layer_norm(x, w, b, eps=1e-5):
    mu = x.mean(-1, keepdims=True)
    var = ((x - mu) ** 2).mean(-1, keepdims=True)
    return (x - mu) / np.sqrt(var + eps) * w + b


def invariants(ori_grid, rel_pos):
    """-> dists [E,1], attr [E,O,2], fiber_attr [O,O,1]."""
    dists = np.sqrt((rel_pos ** 2).sum(-1, keepdims=True))
    r = rel_pos[:, None, :]
    oa = ori_grid[None, :, :]
    ob = ori_grid[:, None, :]
    inv1 = (r * oa).sum(-1, keepdims=True)
    inv2 = np.sqrt(((r - inv1 * oa) ** 2).sum(-1, keepdims=True))
    inv3 = (oa * ob).sum(-1, keepdims=True)
    return dists, np.concatenate([inv1, inv2], -1), inv3


def forward(p, x, vec, edge_index, rel_pos, ori_grid, num_layers, degree=3, multiple_readouts=True,
            out_scalar=0, out_vec=2):
    """x [V, Cs] scalars (mass), vec [V, Cv, 3]; returns [V, out_vec*3]."""
    src, dst = edge_index
    V = x.shape[0]
    O = ori_grid.shape[0]
    # lift to the fibre bundle: [V, O, Cs + Cv]
    xs = np.repeat(x[:, None, :], O, axis=1)
    xv = np.einsum("bcd,nd->bnc", vec, ori_grid)
    f = np.concatenate([xs, xv], -1)
    dists, attr, fiber_attr = invariants(ori_grid, rel_pos)
    kb = gelu(lin(p, "model.basis_fn.3", gelu(lin(p, "model.basis_fn.1", poly_features(attr, degree)))))
    kb = kb * np.ones_like(dists)[:, :, None]            # PolynomialCutoff(None) = 1
    fkb = gelu(lin(p, "model.fiber_basis_fn.3", gelu(lin(p, "model.fiber_basis_fn.1", poly_features(fiber_attr, degree)))))
    h = lin(p, "model.x_embedder", f, bias=False)
    readouts = []
    for i in range(num_layers):
        pre = f"model.interaction_layers.{i}."
        inp = h
        k = lin(p, pre + "conv.kernel", kb, bias=False)              # [E, O, C]
        x1 = np.zeros_like(h)
        np.add.at(x1, dst, k * h[src])                                # aggr add at edge_index[1]
        fk = lin(p, pre + "conv.fiber_kernel", fkb, bias=False)      # [O, O, C]
        x2 = np.einsum("boc,opc->bpc", x1, fk) / fk.shape[-2]
        y = x2 + p[pre + "conv.bias"]
        y = layer_norm(y, p[pre + "norm.weight"], p[pre + "norm.bias"])
        y = lin(p, pre + "linear_2", gelu(lin(p, pre + "linear_1", y)))
        if (pre + "layer_scale") in p:
            y = p[pre + "layer_scale"] * y
        h = y + inp
        if multiple_readouts or i == num_layers - 1:
            readouts.append(lin(p, f"model.read_out_layers.{i}", h))
    readout = sum(readouts) / len(readouts)
    rv = readout[..., out_scalar:out_scalar + out_vec]
    vecs = np.einsum("bnc,nd->bcd", rv, ori_grid) / O
    return vecs.reshape(V, -1)
