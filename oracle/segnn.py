"""numpy fp64 restatement of the reference SEGNN forward — TEST ORACLE ONLY.

Follows, line by line:
* O3TensorProduct / O3TensorProductSwishGate  models/segnn/o3_building_blocks.py:10-203
* O3Transform                                   models/segnn/o3_building_blocks.py:225-278
* SEGNN.__init__/forward, catch_isolated_nodes  models/segnn/segnn.py:17-189
* SEGNNLayer message / update / propagate       models/segnn/segnn.py:192-304
* WeightBalancedIrreps                          models/balanced_irreps.py:51-85
with e3nn semantics from oracle/e3nn_lite.py (parity vs e3nn UNPINNED).

Weights are taken from a flat ``{state_dict key: ndarray}`` dict whose keys are
the reference's own state_dict keys (e.g. ``layers.0.message_layer_1.tp.weight``).
"""
from __future__ import annotations

import math

import numpy as np

from .e3nn_lite import (FullyConnectedTP, Irreps, batch_norm, gate,
                        spherical_harmonics_l1)


def weight_balanced_irreps(hidden_features: int, irreps_in2: Irreps, lmax: int) -> Irreps:
    """models/balanced_irreps.py:51-85 (sh=True)."""
    target = FullyConnectedTP(Irreps(f"{hidden_features}x0e"), "1x0e", Irreps(f"{hidden_features}x0e")).weight_numel
    n = 1
    while True:
        ir1 = (Irreps.spherical_harmonics(lmax) * n).sort()[0].simplify()
        if FullyConnectedTP(ir1, irreps_in2, ir1).weight_numel >= target:
            return ir1
        n += 1


class O3TP:
    """O3TensorProduct (tp_rescale=True): e3nn FCTP, then out /= sqrt_k
    (sqrt_k = 1/sqrt(fan_in) per output slice), then + biases on 0e slices."""

    def __init__(self, irreps_in1, irreps_out, irreps_in2=None):
        self.irreps_in1 = Irreps(irreps_in1)
        self.irreps_out = Irreps(irreps_out)
        self.irreps_in2 = Irreps("1x0e") if irreps_in2 is None else Irreps(irreps_in2)
        self.has_in2 = irreps_in2 is not None
        self.tp = FullyConnectedTP(self.irreps_in1, self.irreps_in2, self.irreps_out)
        self.sqrt_k_correction = np.zeros(self.irreps_out.dim)
        for io, sl in enumerate(self.irreps_out.slices()):
            if io in self.tp.fan_in:
                self.sqrt_k_correction[sl] = 1.0 / math.sqrt(self.tp.fan_in[io])
        self.bias_idx = np.concatenate(
            [np.arange(sl.start, sl.stop) for (m, ir), sl in zip(self.irreps_out, self.irreps_out.slices()) if ir.l == 0]
            or [np.zeros(0, dtype=np.int64)]).astype(np.int64)

    def num_weights(self):
        return self.tp.weight_numel + len(self.bias_idx)

    def __call__(self, p, prefix, x1, x2=None):
        if x2 is None:
            x2 = np.ones((x1.shape[0], 1), dtype=x1.dtype)
        out = self.tp(x1, x2, p[prefix + "tp.weight"])
        out = out / self.sqrt_k_correction.astype(out.dtype)
        if len(self.bias_idx):
            out[:, self.bias_idx] += p[prefix + "biases"]
        return out


class O3TPGate(O3TP):
    def __init__(self, irreps_in1, irreps_out, irreps_in2=None):
        irreps_out = Irreps(irreps_out)
        scalars = Irreps([irreps_out[0]])
        gates = Irreps(f"{irreps_out.num_irreps - scalars.num_irreps}x0e")
        gated = Irreps(list(irreps_out[1:]))
        irreps_g = (scalars + gates + gated).simplify()
        super().__init__(irreps_in1, irreps_g, irreps_in2)
        self.n_scalars, self.n_gates, self.gated = scalars.num_irreps, gates.num_irreps, gated

    def __call__(self, p, prefix, x1, x2=None):
        out = super().__call__(p, prefix, x1, x2)
        return gate(out, self.n_scalars, self.n_gates, self.gated)


def o3_transform(pos, vel, mass, edge_index, lmax_attr=1):
    """O3Transform.__call__ (o3_building_blocks.py:231-278); force input unused.
    Returns (x, edge_attr, node_attr, additional_message_features)."""
    assert lmax_attr == 1
    src, dst = edge_index
    V = pos.shape[0]
    prod_mass = mass[src] * mass[dst]
    rel_pos = pos[src] - pos[dst]
    edge_dist = np.sqrt((rel_pos ** 2).sum(1, keepdims=True))
    edge_attr = spherical_harmonics_l1(rel_pos)
    vel_emb = spherical_harmonics_l1(vel)
    # torch_scatter.scatter(reduce="mean") at edge_index[1]
    acc = np.zeros((V, edge_attr.shape[1]), dtype=pos.dtype)
    cnt = np.zeros((V, 1), dtype=pos.dtype)
    np.add.at(acc, dst, edge_attr)
    np.add.at(cnt, dst, 1.0)
    node_attr = acc / np.maximum(cnt, 1.0) + vel_emb
    vel_abs = np.sqrt((vel ** 2).sum(1, keepdims=True))
    mean_pos = pos.mean(1, keepdims=True)            # NOTE: mean over xyz (reference quirk)
    x = np.concatenate([pos - mean_pos, vel, vel_abs], 1)
    amf = np.concatenate([edge_dist, prod_mass], -1)
    return x, edge_attr, node_attr, amf


class SEGNNOracle:
    """SEGNN(task="node", norm="batch") as built by create_model
    (utils/utils_train.py:56-62): input 2x1o+1x0e, output 2x1o, additional
    message irreps 2x0e, node/edge attrs = SH(lmax_attr)."""

    def __init__(self, hidden_features=64, lmax_h=1, lmax_attr=1, num_layers=4,
                 input_irreps="2x1o+1x0e", output_irreps="2x1o", additional_message_irreps="2x0e"):
        self.num_layers = num_layers
        self.attr_irreps = Irreps.spherical_harmonics(lmax_attr)
        self.hidden_irreps = weight_balanced_irreps(hidden_features, self.attr_irreps, lmax_h)
        h, a = self.hidden_irreps, self.attr_irreps
        amf = Irreps(additional_message_irreps)
        self.embedding = O3TP(Irreps(input_irreps), h, a)
        msg_in = (h + h + amf).simplify()
        upd_in = (h + h).simplify()
        self.ml1 = O3TPGate(msg_in, h, a)
        self.ml2 = O3TPGate(h, h, a)
        self.ul1 = O3TPGate(upd_in, h, a)
        self.ul2 = O3TP(h, h, a)
        self.pre_pool1 = O3TPGate(h, h, a)
        self.pre_pool2 = O3TP(h, Irreps(output_irreps), a)

    def param_shapes(self):
        """{state_dict key: shape} for every learnable parameter / BN buffer."""
        shapes = {}

        def tp(prefix, m):
            shapes[prefix + "tp.weight"] = (m.tp.weight_numel,)
            if len(m.bias_idx):
                shapes[prefix + "biases"] = (len(m.bias_idx),)

        def bn(prefix):
            n_s = sum(m for m, ir in self.hidden_irreps if ir.is_scalar())
            shapes[prefix + "weight"] = (self.hidden_irreps.num_irreps,)
            shapes[prefix + "bias"] = (n_s,)
            shapes[prefix + "running_mean"] = (n_s,)
            shapes[prefix + "running_var"] = (self.hidden_irreps.num_irreps,)

        tp("embedding_layer.", self.embedding)
        for i in range(self.num_layers):
            tp(f"layers.{i}.message_layer_1.", self.ml1)
            tp(f"layers.{i}.message_layer_2.", self.ml2)
            tp(f"layers.{i}.update_layer_1.", self.ul1)
            tp(f"layers.{i}.update_layer_2.", self.ul2)
            bn(f"layers.{i}.feature_norm.")
            bn(f"layers.{i}.message_norm.")
        tp("pre_pool1.", self.pre_pool1)
        tp("pre_pool2.", self.pre_pool2)
        return shapes

    def num_params(self):
        return sum(int(np.prod(s)) for k, s in self.param_shapes().items() if "running" not in k)

    def forward(self, p, x, edge_index, edge_attr, node_attr, amf, training=True):
        """Returns (out[V, 6], updated {running stat key: array}).  ``p`` is not
        mutated; train-mode BatchNorm uses batch statistics (the reference
        rollout never calls model.eval())."""
        node_attr = node_attr.copy()
        node_attr[:, 0] = 1.0                                    # catch_isolated_nodes
        src, dst = edge_index
        V = x.shape[0]
        new_stats = {}
        h = self.embedding(p, "embedding_layer.", x, node_attr)
        for i in range(self.num_layers):
            pre = f"layers.{i}."
            # message(x_i = x[dst], x_j = x[src])
            inp = np.concatenate([h[dst], h[src], amf], -1)
            m = self.ml1(p, pre + "message_layer_1.", inp, edge_attr)
            m = self.ml2(p, pre + "message_layer_2.", m, edge_attr)
            key = pre + "message_norm."
            m, rm, rv = batch_norm(m, self.hidden_irreps, p[key + "weight"], p[key + "bias"],
                                   p[key + "running_mean"], p[key + "running_var"], training)
            new_stats[key + "running_mean"], new_stats[key + "running_var"] = rm, rv
            agg = np.zeros((V, m.shape[1]), dtype=m.dtype)
            np.add.at(agg, dst, m)                               # aggr="add" at edge_index[1]
            # update
            u = self.ul1(p, pre + "update_layer_1.", np.concatenate([h, agg], -1), node_attr)
            u = self.ul2(p, pre + "update_layer_2.", u, node_attr)
            h = h + u
            key = pre + "feature_norm."
            h, rm, rv = batch_norm(h, self.hidden_irreps, p[key + "weight"], p[key + "bias"],
                                   p[key + "running_mean"], p[key + "running_var"], training)
            new_stats[key + "running_mean"], new_stats[key + "running_var"] = rm, rv
        h = self.pre_pool1(p, "pre_pool1.", h, node_attr)
        out = self.pre_pool2(p, "pre_pool2.", h, node_attr)
        return out, new_stats


def init_params(model: SEGNNOracle, seed: int = 0):
    """Independent (numpy) init with the reference's ranges:
    U(-1/sqrt(fan_in), 1/sqrt(fan_in)) per output slice; BN weight 1, bias 0,
    running mean 0, running var 1 (o3_building_blocks.py:82-116)."""
    rng = np.random.default_rng(seed)
    p = {}
    for key, shape in model.param_shapes().items():
        if key.endswith("running_mean") or key.endswith(".bias") and "norm" in key:
            p[key] = np.zeros(shape)
        elif key.endswith("running_var") or (key.endswith(".weight") and "norm" in key):
            p[key] = np.ones(shape)
        else:
            p[key] = rng.uniform(-0.1, 0.1, size=shape)
    return p
