"""numpy restatement of the self-feed rollout loop
(helper_scripts/infer_self_feed.py:99-211) — TEST ORACLE ONLY.

``step_fn(model_type, loc, vel, force, mass) -> pred[V, 6]`` builds the graph the
way the reference's per-model branch does (lines 115-170) and runs the oracle
forward; ``rollout`` then applies lines 182-194 (target "pos_dt+vel")."""
from __future__ import annotations

import numpy as np

from . import egnn_mc as egnn_oracle
from . import ponita as ponita_oracle
from .graph import build_graph_with_knn
from .segnn import o3_transform


def segnn_step(model, params, training=True, lmax_attr=1, num_neighbors=None):
    """SEGNN branch (lines 115-130).  BatchNorm running stats are updated in
    ``params`` after every step, as the train-mode reference module does.
    ``num_neighbors``: the kNN graph of each frame (None: N - 1, fully connected)."""
    def f(loc, vel, force, mass, B, N):
        ei = build_graph_with_knn(loc, B, N, N - 1 if num_neighbors is None else num_neighbors)
        x, ea, na, amf = o3_transform(loc, vel, mass, ei, lmax_attr)
        out, stats = model.forward(params, x, ei, ea, na, amf, training=training)
        params.update(stats)
        return out
    return f


def ponita_step(params, ori_grid, num_layers, num_neighbors=None):
    """PONITA branch (lines 131-147): x = mass, vec = vel[:, None], rel_pos."""
    def f(loc, vel, force, mass, B, N):
        ei = build_graph_with_knn(loc, B, N, N - 1 if num_neighbors is None else num_neighbors)
        rel = loc[ei[0]] - loc[ei[1]]
        return ponita_oracle.forward(params, mass, vel[:, None, :], ei, rel, ori_grid, num_layers)
    return f


def egnn_mc_step(params, num_layers, **kw):
    """EGNN-MC branch (lines 161-170) through EgnnMcNBodyDataLoader.preprocess_batch."""
    def f(loc, vel, force, mass, B, N):
        ei = build_graph_with_knn(loc, B, N, N - 1)
        x, ea = egnn_oracle.preprocess(loc, vel, mass, ei)
        return egnn_oracle.forward(params, x, loc, vel, ei, ea, num_layers, **kw)
    return f


def rollout(step_fn, loc0, vel0, force0, mass0, num_steps, target="pos_dt+vel"):
    """loc0/vel0/force0 [B,N,3], mass0 [B,N,1]; returns (loc_pred, vel_pred)
    each [B, num_steps, N, 3] with frame 0 = the initial state."""
    B, N, D = loc0.shape
    locs, vels = [loc0], [vel0]
    force, mass = force0, mass0
    for _ in range(num_steps - 1):
        loc, vel = locs[-1], vels[-1]
        pred = step_fn(loc.reshape(B * N, D), vel.reshape(B * N, D), force.reshape(B * N, D),
                       mass.reshape(B * N, 1), B, N)
        pl = pred[..., :3].reshape(B, N, D)
        pv = pred[..., 3:].reshape(B, N, D)
        if target == "pos_dt+vel":
            pl = loc + pl
        locs.append(pl)
        vels.append(pv)
        force = np.zeros_like(pl)
    return np.stack(locs, 1), np.stack(vels, 1)
