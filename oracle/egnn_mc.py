"""numpy restatement of the EGNN-MC path — TEST ORACLE ONLY.

* EgnnMcNBodyDataLoader.preprocess_batch  dataloaders/egnn_mc_n_body_dataloader.py:8-56
* _EGNNMessageBlock                       models/egnn_mc/egnn_mc.py:45-186
* _VectorHead / EGNNMultiChannel.forward  models/egnn_mc/egnn_mc.py:189-295
Parameters come from a ``{state_dict key: ndarray}`` dict with the reference's keys
(nn.Linear weights are [out, in])."""
from __future__ import annotations

import numpy as np


def silu(x):
    return x / (1.0 + np.exp(-x))


def _act(name):
    if name == "silu":
        return silu
    if name == "relu":
        return lambda x: np.maximum(x, 0)
    if name in ("leaky_relu", "lrelu"):
        return lambda x: np.where(x > 0, x, 0.2 * x)
    raise ValueError(name)


def linear(p, key, x, bias=True):
    y = x @ p[key + ".weight"].T
    if bias and (key + ".bias") in p:
        y = y + p[key + ".bias"]
    return y


def segment_mean(data, seg, n):
    out = np.zeros((n,) + data.shape[1:], dtype=data.dtype)
    cnt = np.zeros((n,) + data.shape[1:], dtype=data.dtype)
    np.add.at(out, seg, data)
    np.add.at(cnt, seg, 1.0)
    return out / np.maximum(cnt, 1.0)


def preprocess(pos, vel, mass, edge_index):
    """Returns node x [V,2] = [|vel|, mass] and edge_attr [E,4] =
    [m_r m_c, vel_r.d, vel_c.d, |d|^2] with d = pos[row]-pos[col] normalised by
    max(|d|, 1e-12)."""
    row, col = edge_index
    speed = np.sqrt((vel ** 2).sum(-1, keepdims=True))
    x = np.concatenate([speed, mass], -1)
    ev = pos[row] - pos[col]
    d2 = (ev ** 2).sum(-1, keepdims=True)
    direction = ev / np.maximum(np.sqrt(d2), 1e-12)
    proj_r = (vel[row] * direction).sum(-1, keepdims=True)
    proj_c = (vel[col] * direction).sum(-1, keepdims=True)
    mp = mass[row] * mass[col]
    return x, np.concatenate([mp, proj_r, proj_c, d2], -1)


def forward(p, x, pos, vel, edge_index, edge_attr, num_layers, n_targets=2,
            activation="silu", coords_weight=1.0, recurrent=True, norm_diff=True, tanh=True):
    act = _act(activation)
    row, col = edge_index
    V = x.shape[0]
    h = linear(p, "embedding", x)
    coord = pos.copy()
    for i in range(num_layers):
        pre = f"layers.{i}."
        diff = coord[row] - coord[col]
        radial = (diff ** 2).sum(1, keepdims=True)
        if norm_diff:
            diff = diff / np.maximum(np.sqrt(radial), 1.0)
        e_in = np.concatenate([h[row], h[col], radial, edge_attr], -1)
        ef = act(linear(p, pre + "edge_mlp.0", e_in))
        ef = act(linear(p, pre + "edge_mlp.2", ef))
        c = act(linear(p, pre + "coord_mlp.0", ef))
        c = linear(p, pre + "coord_mlp.2", c, bias=False)          # [E, 1]
        if tanh:
            c = np.tanh(c)
        trans = np.clip(diff * c, -100.0, 100.0)
        coord = coord + segment_mean(trans, row, V) * coords_weight
        cv = act(linear(p, pre + "coord_mlp_vel.0", h))
        cv = linear(p, pre + "coord_mlp_vel.2", cv)                 # [V, 1]
        coord = coord + cv * vel
        agg = segment_mean(ef, row, V)
        nout = act(linear(p, pre + "node_mlp.0", np.concatenate([h, agg], -1)))
        nout = linear(p, pre + "node_mlp.2", nout)
        h = h + nout if recurrent else nout
    head_in = np.concatenate([h, coord - pos, vel], -1)
    outs = []
    for t in range(n_targets):
        pre = f"heads.{t}.net."
        y = act(linear(p, pre + "0", head_in))
        y = act(linear(p, pre + "2", y))
        outs.append(linear(p, pre + "4", y))
    return np.concatenate(outs, -1)
