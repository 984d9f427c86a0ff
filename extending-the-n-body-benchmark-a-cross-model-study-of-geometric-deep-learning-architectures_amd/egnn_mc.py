"""EGNNMultiChannel — drop-in for models/egnn_mc/egnn_mc.py with a HIP forward.

Module tree, parameter names/shapes and initialisation order follow the
reference (egnn_mc.py:45-306), so ``torch.manual_seed(s)`` gives the same
weights and reference checkpoints load.  ``forward(graph)`` takes the rollout /
dataloader graph (pos, vel, mass, fully-connected edge_index) and runs the
preprocessing of dataloaders/egnn_mc_n_body_dataloader.py:8-56 plus the model
in libnbx (csrc/egnn.hip); ``rollout`` runs the self-feed loop device-resident.
"""
from __future__ import annotations

from typing import Sequence

import warnings

import torch
from torch import nn

from . import _lib
from .train_dispatch import use_training_path

__all__ = ["EGNNMultiChannel"]


def _make_activation(name: str):
    name = name.lower()
    if name == "silu":
        return nn.SiLU
    if name == "relu":
        return nn.ReLU
    if name in {"leaky_relu", "lrelu"}:
        return lambda: nn.LeakyReLU(negative_slope=0.2)
    raise ValueError(f"Unsupported activation '{name}'.")


class _EGNNMessageBlock(nn.Module):
    """egnn_mc.py:45-130 (parameter container; the arithmetic runs in csrc/egnn.hip)."""

    def __init__(self, node_input_dim, node_output_dim, hidden_edge_dim, hidden_node_dim, hidden_coord_dim, *,
                 edge_attr_dim=0, act_factory=nn.SiLU, coords_weight=1.0, recurrent=True, attention=False,
                 norm_diff=False, tanh=False, num_vectors_in=1, num_vectors_out=1):
        super().__init__()
        self.coords_weight, self.recurrent, self.attention = coords_weight, recurrent, attention
        self.norm_diff, self.tanh = norm_diff, tanh
        self.num_vectors_in, self.num_vectors_out = num_vectors_in, num_vectors_out
        edge_input_dim = node_input_dim * 2 + num_vectors_in + edge_attr_dim
        self.edge_mlp = nn.Sequential(nn.Linear(edge_input_dim, hidden_edge_dim), act_factory(),
                                      nn.Linear(hidden_edge_dim, hidden_edge_dim), act_factory())
        self.node_mlp = nn.Sequential(nn.Linear(hidden_edge_dim + node_input_dim, hidden_node_dim), act_factory(),
                                      nn.Linear(hidden_node_dim, node_output_dim))
        coord_layers = [nn.Linear(hidden_edge_dim, hidden_coord_dim), act_factory(),
                        nn.Linear(hidden_coord_dim, num_vectors_in * num_vectors_out, bias=False)]
        nn.init.xavier_uniform_(coord_layers[-1].weight, gain=0.001)
        if tanh:
            coord_layers.append(nn.Tanh())
        self.coord_mlp = nn.Sequential(*coord_layers)
        self.coord_mlp_vel = nn.Sequential(nn.Linear(node_input_dim, hidden_coord_dim), act_factory(),
                                           nn.Linear(hidden_coord_dim, num_vectors_in * num_vectors_out))
        if attention:
            self.att_mlp = nn.Sequential(nn.Linear(hidden_edge_dim, 1), nn.Sigmoid())


class _VectorHead(nn.Module):
    def __init__(self, input_dim, hidden_dim, act_factory):
        super().__init__()
        self.net = nn.Sequential(nn.Linear(input_dim, hidden_dim), act_factory(), nn.Linear(hidden_dim, hidden_dim),
                                 act_factory(), nn.Linear(hidden_dim, 3))


class EGNNMultiChannel(nn.Module):
    """EGNN variant with learnable vector heads for multiple targets (egnn_mc.py:211-306)."""

    def __init__(self, *, node_input_dim: int = 2, edge_attr_dim: int = 3, hidden_node_dim: int = 128,
                 hidden_edge_dim: int = 128, hidden_coord_dim: int = 128, num_layers: int = 4,
                 target_names: Sequence[str] | None = None, activation: str = "silu", coords_weight: float = 1.0,
                 recurrent: bool = True, norm_diff: bool = False, tanh: bool = False, device="cpu"):
        super().__init__()
        if target_names is None or len(target_names) == 0:
            raise ValueError("EGNNMultiChannel requires at least one target.")
        self.device = torch.device(device)
        self.target_names = tuple(target_names)
        self.hidden_node_dim, self.num_layers = hidden_node_dim, num_layers
        self.activation, self.coords_weight, self.recurrent = activation, coords_weight, recurrent
        self.norm_diff, self.use_tanh = norm_diff, tanh
        act_factory = _make_activation(activation)
        self.embedding = nn.Linear(node_input_dim, hidden_node_dim)
        self.layers = nn.ModuleList([
            _EGNNMessageBlock(hidden_node_dim, hidden_node_dim, hidden_edge_dim, hidden_node_dim, hidden_coord_dim,
                              edge_attr_dim=edge_attr_dim, act_factory=act_factory, coords_weight=coords_weight,
                              recurrent=recurrent, attention=False, norm_diff=norm_diff, tanh=tanh)
            for _ in range(num_layers)])
        head_input_dim = hidden_node_dim + 6
        self.heads = nn.ModuleList([_VectorHead(head_input_dim, hidden_node_dim, act_factory)
                                    for _ in self.target_names])
        native = (activation == "silu" and node_input_dim == 2 and edge_attr_dim == 4
                  and hidden_node_dim == hidden_edge_dim == hidden_coord_dim and hidden_node_dim % 4 == 0
                  and hidden_node_dim <= 128 and len(self.target_names) <= 2)
        self._native_reason = None if native else (
            "native EGNN-MC needs SiLU, node_input_dim 2, edge_attr_dim 4, equal hidden dims (<=128, %4), <=2 heads")
        self._packed = None
        self._ws = None
        self.to(self.device)

    def get_serializable_attributes(self):
        return {"hidden_node_dim": self.hidden_node_dim, "num_layers": self.num_layers,
                "target_names": list(self.target_names), "num_params": sum(p.numel() for p in self.parameters())}

    def get_model_size(self):
        return self.hidden_node_dim

    # ------------------------------------------------------------ packing
    def _param_version(self):
        return tuple((p.data_ptr(), p._version) for p in self.parameters())

    def packed_matrices(self, device, dtype=torch.float32):
        """nn.Linear weights [out][in] with each input segment zero-padded to a
        multiple of 32 columns (include/nbx.h, EGNN-MC section)."""
        H = self.hidden_node_dim
        kp = (H + 31) // 32 * 32
        f = dict(device=device, dtype=dtype)

        def pad_cols(w, segs):
            """segs: list of (width, padded width) covering w's columns in order."""
            out, c = [], 0
            for width, padded in segs:
                part = w[:, c:c + width].to(**f)
                out.append(torch.nn.functional.pad(part, (0, padded - width)))
                c += width
            return torch.cat(out, 1).contiguous()

        def vec(t):
            return t.detach().to(**f).contiguous()

        P = {"emb_t": pad_cols(self.embedding.weight.detach(), [(2, 32)]), "emb_b": vec(self.embedding.bias)}
        for i, L in enumerate(self.layers):
            p = f"layers.{i}."
            P[p + "e0_t"] = pad_cols(L.edge_mlp[0].weight.detach(), [(H, kp), (H, kp), (5, 32)])
            P[p + "e0_b"] = vec(L.edge_mlp[0].bias)
            P[p + "e1_t"] = pad_cols(L.edge_mlp[2].weight.detach(), [(H, kp)])
            P[p + "e1_b"] = vec(L.edge_mlp[2].bias)
            P[p + "c0_t"] = pad_cols(L.coord_mlp[0].weight.detach(), [(H, kp)])
            P[p + "c0_b"] = vec(L.coord_mlp[0].bias)
            P[p + "c1_w"] = vec(L.coord_mlp[2].weight.reshape(-1))
            P[p + "v0_t"] = pad_cols(L.coord_mlp_vel[0].weight.detach(), [(H, kp)])
            P[p + "v0_b"] = vec(L.coord_mlp_vel[0].bias)
            P[p + "v1_w"] = vec(L.coord_mlp_vel[2].weight.reshape(-1))
            P[p + "v1_b"] = vec(L.coord_mlp_vel[2].bias)
            P[p + "n0_t"] = pad_cols(L.node_mlp[0].weight.detach(), [(H, kp), (H, kp)])
            P[p + "n0_b"] = vec(L.node_mlp[0].bias)
            P[p + "n1_t"] = pad_cols(L.node_mlp[2].weight.detach(), [(H, kp)])
            P[p + "n1_b"] = vec(L.node_mlp[2].bias)
        for t, head in enumerate(self.heads):
            p = f"heads.{t}."
            P[p + "w0_t"] = pad_cols(head.net[0].weight.detach(), [(H, kp), (6, 32)])
            P[p + "b0"] = vec(head.net[0].bias)
            P[p + "w1_t"] = pad_cols(head.net[2].weight.detach(), [(H, kp)])
            P[p + "b1"] = vec(head.net[2].bias)
            P[p + "w2_t"] = pad_cols(head.net[4].weight.detach(), [(H, kp)])
            P[p + "b2"] = vec(head.net[4].bias)
        P["persist_blob"] = self.persist_blob(device)
        return P

    def persist_blob(self, device, differentiable: bool = False):
        """The input-major weight blob of the persistent per-system kernel (include/nbx.h).
        ``differentiable``: built from the parameters with autograd-tracked ops, so a gradient
        of the blob (nbx_egnn_train_backward) flows back to every parameter."""
        src = (lambda w: w) if differentiable else (lambda w: w.detach())
        return self._blob_from(src, dict(device=device, dtype=torch.float32))

    def _blob_from(self, src, f):
        H = self.hidden_node_dim

        def t(w, rows=None, cols=None):          # nn.Linear [out][in] -> [in][out], zero-padded
            x = src(w).to(**f).T
            r, c = rows or x.shape[0], cols or x.shape[1]
            return torch.nn.functional.pad(x, (0, c - x.shape[1], 0, r - x.shape[0])).reshape(-1)

        def v(b, n=None):
            x = src(b).to(**f).reshape(-1)
            return torch.nn.functional.pad(x, (0, (n or x.numel()) - x.numel()))

        parts = [t(self.embedding.weight), v(self.embedding.bias)]
        for L in self.layers:
            parts += [t(L.edge_mlp[0].weight, rows=2 * H + 8), v(L.edge_mlp[0].bias), t(L.edge_mlp[2].weight),
                      v(L.edge_mlp[2].bias), t(L.coord_mlp[0].weight), v(L.coord_mlp[0].bias),
                      v(L.coord_mlp[2].weight), t(L.coord_mlp_vel[0].weight), v(L.coord_mlp_vel[0].bias),
                      v(L.coord_mlp_vel[2].weight), v(L.coord_mlp_vel[2].bias, 4), t(L.node_mlp[0].weight),
                      v(L.node_mlp[0].bias), t(L.node_mlp[2].weight), v(L.node_mlp[2].bias)]
        for head in self.heads:
            parts += [t(head.net[0].weight, rows=H + 8), v(head.net[0].bias), t(head.net[2].weight),
                      v(head.net[2].bias), t(head.net[4].weight, cols=4), v(head.net[4].bias, 4)]
        blob = torch.cat(parts).contiguous()
        L_, nh = len(self.layers), len(self.heads)
        assert blob.numel() == 3 * H + L_ * (8 * H * H + 16 * H + 4) + nh * (2 * H * H + 14 * H + 4)
        return blob

    def pack_weights(self, device):
        P = self.packed_matrices(device)
        W = _lib.EgnnWeights()
        W.hidden, W.num_layers, W.num_heads = self.hidden_node_dim, self.num_layers, len(self.heads)
        W.recurrent, W.norm_diff, W.use_tanh = int(self.recurrent), int(self.norm_diff), int(self.use_tanh)
        W.coords_weight = float(self.coords_weight)
        W.emb_t, W.emb_b = P["emb_t"].data_ptr(), P["emb_b"].data_ptr()
        W.persist_blob = P["persist_blob"].data_ptr()
        for i in range(self.num_layers):
            L = W.layers[i]
            for name, _ in L._fields_:
                if name == "v1_b":
                    L.v1_b = float(P[f"layers.{i}.v1_b"].item())
                else:
                    setattr(L, name, P[f"layers.{i}.{name}"].data_ptr())
        for t in range(len(self.heads)):
            for name, _ in W.heads[t]._fields_:
                setattr(W.heads[t], name, P[f"heads.{t}.{name}"].data_ptr())
        self._packed = (self._param_version(), W, P)
        return W

    def invalidate_weights(self):
        """Drop the packed inference weights.  Call after updating the parameters in a way that does
        not bump their version counters -- e.g. replays of a captured training step (HIP graph), whose
        optimizer writes the parameters in place on the device."""
        self._packed = None
        return self

    def _weights(self, device):
        if self._native_reason:
            raise NotImplementedError(self._native_reason)
        if self._packed is None or self._packed[0] != self._param_version():
            self.pack_weights(device)
        return self._packed[1]

    def _workspace(self, B, N, device):
        n = _lib.c_sz()
        _lib.check(_lib.lib().nbx_egnn_workspace_bytes(B, N, self.hidden_node_dim, n), "egnn workspace")
        if self._ws is None or self._ws.numel() < n.value or self._ws.device != device:
            self._ws = torch.empty(n.value, dtype=torch.uint8, device=device)
        return self._ws

    # ------------------------------------------------------------ training blob
    def _train_layout(self, device):
        """(params, index, blob_floats): the parameters the blob holds, in a fixed order, and the blob
        position of every element of their flattened concatenation -- persist_blob's layout traced
        once with element ids, so a training step packs the blob with one scatter and maps the blob
        gradient back onto the parameters with one gather."""
        device = torch.device(device)
        cached = getattr(self, "_tlayout", None)
        if cached is not None and cached[0] == device:   # (reset by _apply: .to() / .float() / ...)
            return cached[1:]
        params = list(self.parameters())
        ids, base = {}, 1
        for q in params:
            ids[id(q)] = torch.arange(base, base + q.numel(), dtype=torch.float64).reshape(q.shape)
            base += q.numel()
        tagged = self._blob_from(lambda w: ids[id(w)], dict(device="cpu", dtype=torch.float64)).to(torch.int64)
        pos = torch.nonzero(tagged).reshape(-1)
        elem = tagged[pos] - 1                       # flat parameter element at each blob position
        index = torch.full((base - 1,), -1, dtype=torch.int64)
        index[elem] = pos
        used, off = [], 0
        for q in params:
            sl = index[off:off + q.numel()]
            if bool((sl >= 0).all()):
                used.append((q, sl))
            elif bool((sl >= 0).any()):
                raise RuntimeError("persist blob holds part of a parameter")
            off += q.numel()
        idx = torch.cat([sl for _, sl in used]).to(device)
        self._tlayout = (device, [q for q, _ in used], idx, int(tagged.numel()))
        return self._tlayout[1:]

    def _apply(self, fn, *args, **kwargs):
        self._tlayout = None   # parameters may be replaced
        return super()._apply(fn, *args, **kwargs)

    def _train_weights(self, blob):
        """The weight struct of the training entry points: the model's flags and the blob."""
        W = _lib.EgnnWeights()
        W.hidden, W.num_layers, W.num_heads = self.hidden_node_dim, self.num_layers, len(self.heads)
        W.recurrent, W.norm_diff, W.use_tanh = int(self.recurrent), int(self.norm_diff), int(self.use_tanh)
        W.coords_weight = float(self.coords_weight)
        W.persist_blob = blob.data_ptr()
        return W

    # ------------------------------------------------------------ forward
    def _untrainable_reason(self, N: int):
        """None if the native training step (csrc/egnn_train.hip check_train) covers systems of N
        bodies, else why not: 2 <= N <= 8 within 160 KiB of LDS, hidden % 4 == 0, 1-2 heads."""
        H, E = self.hidden_node_dim, N * (N - 1)
        lds = 2 * E * (2 * H + 8) + 3 * E * H + 10 * N * H + 512 + 16 * E + 32 * N
        if not 2 <= N <= 8:
            return f"systems of N = {N} bodies (the native training step needs 2 <= N <= 8)"
        if H % 4:
            return f"hidden {H} (the native training step needs hidden % 4 == 0)"
        if lds * 4 > 160 * 1024:
            return f"hidden {H} at N = {N} needs {lds * 4} bytes of LDS per system (> 160 KiB)"
        if not 1 <= len(self.heads) <= 2:
            return f"{len(self.heads)} output heads (the native training step needs 1 or 2)"
        return None

    def _trainable(self, N: int) -> bool:
        return self._untrainable_reason(N) is None

    def forward(self, graph):
        pos = graph.pos
        device = pos.device
        V = pos.shape[0]
        from .graph import system_layout
        # (graph.nbx_system_size, set by this package's dataloaders for fully-connected graphs, skips
        # the host-side edge_index comparison: a captured training step needs that)
        B, N, fc = system_layout(graph, V, graph.edge_index.shape[1], device)
        knn = None if fc else self._knn_table(graph.edge_index, B, N, device)
        f = lambda t: t.detach().to(device=device, dtype=torch.float32).contiguous()
        mass = getattr(graph, "mass", None)
        m = f(mass.reshape(-1)) if mass is not None else torch.ones(V, device=device)
        p, v = f(pos), f(graph.vel)
        if use_training_path(self):   # train_dispatch.py: autograd on + trainable params
            # training step (trainer.py:233-358): the native forward keeps its activations and
            # loss.backward() runs the native backward (csrc/egnn_train.hip).  Inputs it does not
            # cover raise here, instead of returning an inference result without an autograd graph
            # (whose parameters AdamW would silently skip).
            if self._native_reason:
                raise NotImplementedError(self._native_reason)
            if knn is not None:
                raise NotImplementedError("native EGNN-MC training step: kNN graphs (num_neighbors < N-1) are not "
                                          "supported; the training forward runs fully-connected systems")
            why = self._untrainable_reason(N)
            if why:
                raise NotImplementedError("native EGNN-MC training step: " + why)
            if any(q.dtype == torch.float64 for q in self.parameters()) and not getattr(self, "_warned_f64", False):
                warnings.warn("EGNN-MC native training computes in fp32: float64 parameters (double_precision "
                              "datasets) are cast to fp32 for the step and the gradients cast back", stacklevel=2)
                self._warned_f64 = True
            params, idx, nblob = self._train_layout(device)
            return _EgnnTrainFn.apply(self, idx, nblob, p, v, m, B, N, *params).to(pos.dtype)
        out = torch.empty(V, 3 * len(self.heads), device=device, dtype=torch.float32)
        W = self._weights(device)
        ws = self._workspace(B, N, device)
        if knn is None:
            _lib.check(_lib.lib().nbx_egnn_forward(W, _lib.dev_ptr(p), _lib.dev_ptr(v), _lib.dev_ptr(m), B, N,
                                                   _lib.dev_ptr(out), _lib.dev_ptr(ws), ws.numel(),
                                                   _lib.stream_ptr(device)), "nbx_egnn_forward")
        else:
            k, nbr = knn
            _lib.check(_lib.lib().nbx_egnn_forward_graph(W, _lib.dev_ptr(p), _lib.dev_ptr(v), _lib.dev_ptr(m), B, N,
                                                         k, _lib.dev_ptr(nbr), _lib.dev_ptr(out), _lib.dev_ptr(ws),
                                                         ws.numel(), _lib.stream_ptr(device)),
                       "nbx_egnn_forward_graph")
        return out.to(pos.dtype)

    @staticmethod
    def _knn_table(edge_index, B: int, N: int, device):
        """(k, nbr int32 [B N][k]) of a graph with k edges at every row node, in row order (the kNN
        graphs of build_graph_with_knn, build_fully_connected_graph.py:42-80, which
        egnn_mc_n_body_dataloader.py:21-28 hands the model); nbr holds local column indices.
        EGNN-MC aggregates at row = edge_index[0] (egnn_mc.py:127-128, 142-151), so other graphs
        (ragged degrees) are refused.  (A grad-mode forward on such a graph returns the inference
        result, as for shapes the native training step does not cover.)"""
        V = B * N
        ei = edge_index.to(device)
        E = ei.shape[1]
        k = E // V if V else 0
        msg = ("native EGNN-MC runs the fully-connected graph or k < N-1 edges at every node, grouped by "
               "row = edge_index[0] (build_graph_with_knn's kNN layout)")
        if E != V * k or not 1 <= k < N - 1:
            raise NotImplementedError(msg)
        row, col = ei[0], ei[1]
        if not torch.equal(row, torch.arange(V, device=device, dtype=row.dtype).repeat_interleave(k)):
            raise NotImplementedError(msg)
        local = col - torch.div(row, N, rounding_mode="floor") * N
        if bool(((local < 0) | (local >= N)).any()):
            raise NotImplementedError("native EGNN-MC: edges between systems")
        return k, local.to(torch.int32).contiguous()

    @torch.no_grad()
    def rollout(self, loc, vel, mass, num_frames: int, absolute: bool = False, num_neighbors=None):
        """Device-resident self-feed (infer_self_feed.py:161-194); ``absolute``: pos = pred[:, :3]
        (targets other than "pos_dt+vel") instead of pos += pred[:, :3].  ``num_neighbors``: the
        dataloader's kNN option (egnn_mc_n_body_dataloader.py:13-28): each frame's graph is the kNN
        graph of that frame's positions, built inside the rollout kernel (None / N-1: fully
        connected)."""
        device = loc.device
        B, N, _ = loc.shape
        f = lambda t: t.detach().to(device=device, dtype=torch.float32).contiguous().clone()
        p, v, m = f(loc), f(vel), f(mass.reshape(B * N))
        tp = torch.empty(B, num_frames, N, 3, device=device, dtype=torch.float32)
        tv = torch.empty_like(tp)
        W = self._weights(device)
        ws = self._workspace(B, N, device)
        flags = _lib.ROLLOUT_ABSOLUTE if absolute else 0
        if num_neighbors is None or int(num_neighbors) == N - 1:
            _lib.check(_lib.lib().nbx_egnn_rollout(W, _lib.dev_ptr(p), _lib.dev_ptr(v), _lib.dev_ptr(m), B, N,
                                                   num_frames, flags, _lib.dev_ptr(tp), _lib.dev_ptr(tv),
                                                   _lib.dev_ptr(ws), ws.numel(), _lib.stream_ptr(device)),
                       "nbx_egnn_rollout")
        else:
            _lib.check(_lib.lib().nbx_egnn_rollout_knn(W, _lib.dev_ptr(p), _lib.dev_ptr(v), _lib.dev_ptr(m), B, N,
                                                       num_frames, flags, int(num_neighbors), _lib.dev_ptr(tp),
                                                       _lib.dev_ptr(tv), _lib.dev_ptr(ws), ws.numel(),
                                                       _lib.stream_ptr(device)), "nbx_egnn_rollout_knn")
        return tp, tv


class _EgnnTrainFn(torch.autograd.Function):
    """Native training forward / backward of EGNNMultiChannel (include/nbx.h
    nbx_egnn_train_forward / nbx_egnn_train_backward).  Inputs: the parameters the weight blob
    holds; forward scatters them into the blob (one launch) and runs the native forward, output =
    pred [V, 3 heads]; backward runs the native backward to dL/dblob and gathers it back onto the
    parameters (one launch)."""

    @staticmethod
    def forward(ctx, model, idx, nblob, pos, vel, mass, B, N, *params):
        device = pos.device
        flat = torch.cat([q.detach().reshape(-1).to(torch.float32) for q in params])
        blob = torch.zeros(nblob, device=device, dtype=torch.float32).index_copy_(0, idx, flat)
        W = model._train_weights(blob)
        n = _lib.c_sz()
        _lib.check(_lib.lib().nbx_egnn_train_workspace_bytes(W, B, N, n), "nbx_egnn_train_workspace_bytes")
        ws = torch.empty(n.value, dtype=torch.uint8, device=device)
        out = torch.empty(B * N, 3 * W.num_heads, device=device, dtype=torch.float32)
        _lib.check(_lib.lib().nbx_egnn_train_forward(W, _lib.dev_ptr(pos), _lib.dev_ptr(vel), _lib.dev_ptr(mass), B, N,
                                                     _lib.dev_ptr(out), _lib.dev_ptr(ws), ws.numel(),
                                                     _lib.stream_ptr(device)), "nbx_egnn_train_forward")
        ctx.W, ctx.B, ctx.N, ctx.ws, ctx.blob, ctx.idx = W, B, N, ws, blob, idx
        ctx.shapes = [(q.shape, q.dtype) for q in params]
        ctx.save_for_backward(pos, vel, mass)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        if ctx.ws is None:
            raise RuntimeError("EGNN-MC native training step: backward ran twice through the same forward "
                               "(retain_graph=True is not supported: the activations are released after the "
                               "first backward)")
        pos, vel, mass = ctx.saved_tensors
        device = pos.device
        g = grad_out.detach().to(device=device, dtype=torch.float32).contiguous()
        grad_blob = torch.empty_like(ctx.blob)
        _lib.check(_lib.lib().nbx_egnn_train_backward(ctx.W, _lib.dev_ptr(pos), _lib.dev_ptr(vel), _lib.dev_ptr(mass),
                                                      ctx.B, ctx.N, _lib.dev_ptr(g), _lib.dev_ptr(grad_blob),
                                                      _lib.dev_ptr(ctx.ws), ctx.ws.numel(),
                                                      _lib.stream_ptr(device)), "nbx_egnn_train_backward")
        flat = grad_blob.index_select(0, ctx.idx)
        grads, off = [], 0
        for shape, dtype in ctx.shapes:
            k = shape.numel()
            grads.append(flat[off:off + k].view(shape).to(dtype))
            off += k
        ctx.ws = ctx.blob = None
        return (None,) * 8 + tuple(grads)
