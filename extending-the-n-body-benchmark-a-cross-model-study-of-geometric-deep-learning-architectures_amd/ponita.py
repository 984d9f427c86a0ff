"""PONITA_NBODY — drop-in for models/ponita/ponita_nbody.py with a HIP forward.

Module tree, parameter names and initialisation order follow the reference
(ponita_nbody.py:12-80, models/ponita_pg.py:59-127, nn/conv.py:65-101,
nn/convnext.py:4-16), including the S2 orientation grid drawn by repulsion at
construction (geometry/rotation.py:916-1010, geometry/repulsion.py:31-90) and the
two LazyLinear layers materialised at the first forward, so ``torch.manual_seed(s)``
gives the reference's grid and weights and reference checkpoints load.  Unlike the
reference, the grid is a persistent buffer (``model.ori_grid``): a checkpoint
written here carries it; loading a reference checkpoint (which has none) keeps
the grid of the constructed model, exactly as the reference does.

``forward(graph)`` takes the rollout / dataloader graph (x = mass, vec = vel,
pos, fully-connected edge_index; infer_self_feed.py:131-147,
dataloaders/ponita_n_body_dataloader.py:8-38) and runs the whole model in libnbx
(csrc/ponita.hip).  The first training-mode forward performs the one-time
FiberBundleConv "callibrate" weight rescaling (conv.py:115-117,134-140) from
moments the HIP path returns.  ``rollout`` runs the self-feed loop device-resident.
"""
from __future__ import annotations

import math

import torch
from torch import nn

from . import _lib
from .train_dispatch import use_training_path

__all__ = ["PONITA_NBODY", "PonitaFiberBundle", "uniform_grid_s2"]


# ------------------------------------------------------------------ S2 grid
def _spherical_to_euclid(g):
    x = g.new_empty((*g.shape[:-1], 3))
    beta, gamma = g[..., 0], g[..., 1]
    x[..., 0] = torch.sin(beta) * torch.cos(gamma)
    x[..., 1] = torch.sin(beta) * torch.sin(gamma)
    x[..., 2] = torch.cos(beta)
    return x


def _euclid_to_spherical(x):
    g = x.new_empty((*x.shape[:-1], 2))
    g[..., 0] = torch.acos(x[..., 2])
    g[..., 1] = torch.atan2(x[..., 1], x[..., 0])
    return g


def _geodesic_distance_s2(r1, r2, eps: float = 1e-7):
    return torch.acos(torch.clamp((r1 * r2).sum(-1), -1 + eps, 1 - eps))


def uniform_grid_s2(n: int, steps: int = 100, step_size: float = 0.1, alpha: float = 0.001) -> torch.Tensor:
    """rotation.py:946-1010 with parameterization 'euclidean': a random S2 grid
    (random_s2, rotation.py:916-929) relaxed by Coulomb repulsion under SGD with
    annealed gradient noise (repulsion.py:31-90).  Consumes the global RNG in the
    same order as the reference."""
    x = torch.randn((n, 3))
    grid = _euclid_to_spherical(x / torch.linalg.norm(x, dim=-1, keepdim=True))
    with torch.enable_grad():
        grid.requires_grad = True
        opt = torch.optim.SGD([grid], lr=step_size)
        for epoch in range(steps):
            opt.zero_grad(set_to_none=True)
            e = _spherical_to_euclid(grid)
            dists = _geodesic_distance_s2(e[:, None], e).sort(dim=-1)[0][:, 1:]
            energy = (dists / math.pi) ** (-2)
            energy.mean().backward()
            grid.grad += (steps - epoch) / steps * alpha * torch.randn(grid.grad.shape)
            opt.step()
        grid.requires_grad = False
    return _spherical_to_euclid(grid.detach())


# ------------------------------------------------------------------ modules
class PolynomialFeatures(nn.Module):
    """nn/embedding.py:4-15 (parameter-free; its arithmetic is in po_attr_kernel)."""

    def __init__(self, degree):
        super().__init__()
        self.degree = degree


class FiberBundleConv(nn.Module):
    """nn/conv.py:65-101: separable depth-wise conv parameters + the callibrated flag."""

    def __init__(self, channels, attr_dim):
        super().__init__()
        self.kernel = nn.Linear(attr_dim, channels, bias=False)
        self.fiber_kernel = nn.Linear(attr_dim, channels, bias=False)
        self.bias = nn.Parameter(torch.empty(channels))
        self.bias.data.zero_()
        self.register_buffer("callibrated", torch.tensor(False))


class ConvNext(nn.Module):
    """nn/convnext.py:4-16."""

    def __init__(self, channels, conv, layer_scale=1e-6, widening_factor=4):
        super().__init__()
        self.conv = conv
        self.act_fn = nn.GELU()
        self.linear_1 = nn.Linear(channels, widening_factor * channels)
        self.linear_2 = nn.Linear(widening_factor * channels, channels)
        if layer_scale is not None:
            self.layer_scale = nn.Parameter(torch.ones(channels) * layer_scale)
        else:
            self.register_buffer("layer_scale", None)
        self.norm = nn.LayerNorm(channels)


class PonitaFiberBundle(nn.Module):
    """models/ponita_pg.py:56-127 (fibre-bundle variant, task_level 'node')."""

    def __init__(self, input_dim, hidden_dim, output_dim, num_layers, output_dim_vec=0, radius=None, num_ori=20,
                 basis_dim=None, degree=3, widening_factor=4, layer_scale=None, multiple_readouts=True):
        super().__init__()
        self.output_dim, self.output_dim_vec = output_dim, output_dim_vec
        self.hidden_dim, self.num_ori, self.degree, self.radius = hidden_dim, num_ori, degree, radius
        self.widening_factor = widening_factor
        # PositionOrientationGraph(num_ori) draws the grid at construction (position_orientation_graph.py:31-32)
        self.register_buffer("ori_grid", uniform_grid_s2(num_ori))
        basis_dim = hidden_dim if basis_dim is None else basis_dim
        self.basis_dim = basis_dim
        self.basis_fn = nn.Sequential(PolynomialFeatures(degree), nn.LazyLinear(hidden_dim), nn.GELU(),
                                      nn.Linear(hidden_dim, basis_dim), nn.GELU())
        self.fiber_basis_fn = nn.Sequential(PolynomialFeatures(degree), nn.LazyLinear(hidden_dim), nn.GELU(),
                                            nn.Linear(hidden_dim, basis_dim), nn.GELU())
        self.x_embedder = nn.Linear(input_dim, hidden_dim, False)
        self.interaction_layers = nn.ModuleList()
        self.read_out_layers = nn.ModuleList()
        for i in range(num_layers):
            conv = FiberBundleConv(hidden_dim, basis_dim)
            self.interaction_layers.append(ConvNext(hidden_dim, conv, layer_scale=layer_scale,
                                                    widening_factor=widening_factor))
            if multiple_readouts or i == num_layers - 1:
                self.read_out_layers.append(nn.Linear(hidden_dim, output_dim + output_dim_vec))
            else:
                self.read_out_layers.append(None)

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        # reference checkpoints do not carry the grid: keep the constructed one
        key = prefix + "ori_grid"
        if key not in state_dict:
            state_dict[key] = self.ori_grid
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                                      error_msgs)

    def materialize(self):
        """LazyLinear(hidden) of both basis MLPs, in forward order (basis_fn first),
        initialised on the CPU generator in the model dtype as the reference's first
        forward does (in_features = 14 and 3 for degree 3 and 2 / 1 invariants)."""
        ref = self.x_embedder.weight
        for seq, n_inv in ((self.basis_fn, 2), (self.fiber_basis_fn, 1)):
            lazy = seq[1]
            if isinstance(lazy, nn.modules.lazy.LazyModuleMixin) and lazy.has_uninitialized_params():
                fan_in = sum(n_inv ** k for k in range(1, self.degree + 1))
                lin = nn.Linear(fan_in, lazy.out_features, dtype=ref.dtype)
                seq[1] = lin.to(ref.device)


class PONITA_NBODY(nn.Module):
    """ponita_nbody.py:9-116.  ``forward(graph) -> [B*N, 6]`` (pos_dt | vel)."""

    def __init__(self, lr=1e-3, weight_decay=1e-5, warmup=10, layer_scale=1e-6, train_augm=False, hidden_dim=64,
                 layers=4, radius=None, num_ori=20, basis_dim=128, degree=3, widening_factor=4,
                 multiple_readouts=True, in_channels_scalar=1, in_channels_vec=1, out_channels_scalar=0,
                 out_channels_vec=2):
        super().__init__()
        self.lr, self.weight_decay, self.warmup = lr, weight_decay, warmup
        self.layer_scale, self.train_augm = layer_scale, train_augm
        self.hidden_dim, self.layers, self.radius, self.num_ori = hidden_dim, layers, radius, num_ori
        self.basis_dim, self.degree, self.widening_factor = basis_dim, degree, widening_factor
        self.multiple_readouts = multiple_readouts
        self.in_channels_scalar, self.in_channels_vec = in_channels_scalar, in_channels_vec
        self.out_channels_scalar, self.out_channels_vec = out_channels_scalar, out_channels_vec
        if layer_scale == 0.0:
            layer_scale = None
        self.model = PonitaFiberBundle(in_channels_scalar + in_channels_vec, hidden_dim, out_channels_scalar, layers,
                                       output_dim_vec=out_channels_vec, radius=radius, num_ori=num_ori,
                                       basis_dim=basis_dim, degree=degree, widening_factor=widening_factor,
                                       layer_scale=layer_scale, multiple_readouts=multiple_readouts)
        bd = hidden_dim if basis_dim is None else basis_dim
        native = (in_channels_scalar == 1 and in_channels_vec == 1 and out_channels_scalar == 0
                  and out_channels_vec == 2 and radius is None and degree == 3 and hidden_dim in (32, 64, 128)
                  and bd % 4 == 0 and bd <= 1024 and 1 <= num_ori <= 24 and widening_factor * hidden_dim <= 1024
                  and 1 <= layers <= _lib.PONITA_MAX_LAYERS)
        self._native_reason = None if native else (
            "native PONITA needs x = mass, vec = vel, 2 vector outputs, radius None, degree 3, hidden in "
            "{32, 64, 128}, basis_dim % 4 == 0, num_ori <= 24, widening * hidden <= 1024")
        self._packed = None
        self._ws = None
        # torch.distributed group whose ranks share the one-time calibration (sharded batches: the
        # moments of the whole global batch, as the reference's single process sees them); None = local
        self.calibration_group = None

    def get_serializable_attributes(self):
        return {"lr": self.lr, "weight_decay": self.weight_decay, "warmup": self.warmup,
                "layer_scale": self.layer_scale, "train_augm": self.train_augm, "hidden_dim": self.hidden_dim,
                "layers": self.layers, "radius": self.radius, "num_ori": self.num_ori, "basis_dim": self.basis_dim,
                "degree": self.degree, "widening_factor": self.widening_factor,
                "multiple_readouts": self.multiple_readouts}

    def get_model_size(self):
        return self.hidden_dim

    # ------------------------------------------------------------ packing
    def _param_version(self):
        return tuple((p.data_ptr(), p._version) for p in self.parameters()) + (
            self.model.ori_grid.data_ptr(), self.model.ori_grid._version)

    def packed_matrices(self, device, dtype=torch.float32):
        """nn.Linear weights [out][K] with K zero-padded to a multiple of 32
        (include/nbx.h, PONITA section)."""
        m = self.model
        m.materialize()
        f = dict(device=device, dtype=dtype)
        kp = lambda k: (k + 31) // 32 * 32

        def pad(w):
            w = w.detach().to(**f)
            return nn.functional.pad(w, (0, kp(w.shape[1]) - w.shape[1])).contiguous()

        vec = lambda t: t.detach().to(**f).contiguous()
        P = {"ori_grid": vec(m.ori_grid), "embed_w": vec(m.x_embedder.weight),
             "basis1_t": pad(m.basis_fn[1].weight), "basis1_b": vec(m.basis_fn[1].bias),
             "basis2_t": pad(m.basis_fn[3].weight), "basis2_b": vec(m.basis_fn[3].bias),
             "fbasis1_t": pad(m.fiber_basis_fn[1].weight), "fbasis1_b": vec(m.fiber_basis_fn[1].bias),
             "fbasis2_t": pad(m.fiber_basis_fn[3].weight), "fbasis2_b": vec(m.fiber_basis_fn[3].bias),
             "fiber_t": pad(torch.cat([L.conv.fiber_kernel.weight.detach() for L in m.interaction_layers], 0))}
        for i, (L, R) in enumerate(zip(m.interaction_layers, m.read_out_layers)):
            p = f"layers.{i}."
            P[p + "kernel_t"] = pad(L.conv.kernel.weight)
            P[p + "conv_bias"] = vec(L.conv.bias)
            P[p + "norm_w"], P[p + "norm_b"] = vec(L.norm.weight), vec(L.norm.bias)
            P[p + "lin1_t"], P[p + "lin1_b"] = pad(L.linear_1.weight), vec(L.linear_1.bias)
            P[p + "lin2_t"], P[p + "lin2_b"] = pad(L.linear_2.weight), vec(L.linear_2.bias)
            if L.layer_scale is not None:
                P[p + "layer_scale"] = vec(L.layer_scale)
            if R is not None:
                P[p + "readout_w"], P[p + "readout_b"] = vec(R.weight), vec(R.bias)
        # split-precision (bf16x3) images of the large GEMMs' weights (include/nbx.h "bf16x3
        # images", CW = 32, one sub-tile): fp32-accurate products at 2.7x the fp32 MFMA rate
        for key, name in [("basis2_t", "basis2_img_x3")] + [
                (f"layers.{i}.{k}_t", f"layers.{i}.{k}_img_x3") for i in range(len(m.interaction_layers))
                for k in ("kernel", "lin1", "lin2")]:
            W = P[key]
            if W.shape[0] % 32 == 0:
                P[name] = self.lin_image_x3(W)
                if name.endswith("lin2_img_x3"):   # the row-panel kernel streams K chunks: chunk-major
                    img = P[name]
                    P[name] = img.reshape(img.shape[0], W.shape[1] // 32, -1).transpose(0, 1).contiguous()
        C = m.hidden_dim
        # the kernel-basis MLP as one fused kernel (csrc/ponita.hip po_ffn_kernel FFN_BASIS)
        if C % 32 == 0 and C <= 1024 and m.basis_dim in (64, 128) and P["basis1_t"].shape[1] == 32:
            P["basis_ffn_img_x3"] = self._ffn_image(P["basis1_t"], P["basis2_t"])
            P["basis_ffn_img_h2"], P["basis_ffn_h2_s1inv"], P["basis_ffn_h2_s2inv"] = self._ffn_image_h2(
                P["basis1_t"], P["basis2_t"])
        for i in range(len(m.interaction_layers)):
            p = f"layers.{i}."
            if C in (64, 128) and P[p + "lin1_t"].shape[0] % 32 == 0:
                P[p + "ffn_img_x3"] = self._ffn_image(P[p + "lin1_t"], P[p + "lin2_t"])
                P[p + "ffn_img_h2"], P[p + "ffn_h2_s1inv"], P[p + "ffn_h2_s2inv"] = self._ffn_image_h2(
                    P[p + "lin1_t"], P[p + "lin2_t"])
            Wk = P[p + "kernel_t"]
            if Wk.shape[0] % 32 == 0:   # the spatial conv (LIN_CONV) on fp16x2 (include/nbx.h "fp16x2 images")
                s = self.h2_scale(Wk)
                P[p + "kernel_img_h2"] = self.lin_image_h2(Wk, s)
                P[p + "kernel_h2_sinv"] = torch.tensor(1.0 / s, dtype=torch.float64)
        return P

    @staticmethod
    def h2_scale(*mats):
        from .segnn import SEGNN
        return SEGNN.h2_scale(*mats)

    @classmethod
    def _ffn_image_h2(cls, W1, W2):
        """include/nbx.h nbx_ponita_layer.ffn_img_h2: the _ffn_image slabs with fp16x2 blocks, W1 scaled by
        s1 and W2 by s2 (powers of two, max |W s| in [2^9, 2^10)); returns (image, 1 / s1, 1 / s2)."""
        F, C = W1.shape[0], W2.shape[0]
        nj = F // 32
        s1, s2 = cls.h2_scale(W1), cls.h2_scale(W2[:, :F])
        img1 = cls.lin_image_h2(W1, s1).reshape(nj, -1)
        perm = torch.tensor([32 * j + q for j in range(nj) for q in cls.FFN_PERM], device=W2.device)
        W2p = W2[:, :F][:, perm].contiguous()
        img2 = cls.lin_image_h2(W2p, s2).reshape(C // 32, nj, -1).transpose(0, 1).reshape(nj, -1)
        inv = lambda x: torch.tensor(1.0 / x, dtype=torch.float64)   # exact: powers of two
        return torch.cat([img1, img2], 1).contiguous(), inv(s1), inv(s2)

    @staticmethod
    def lin_image_h2(W, scale):
        """[N][Kp] -> int16 fp16x2 image [N/32][Kp/32][2][2][64][8] of W * scale (include/nbx.h "fp16x2 images")."""
        from .segnn import SEGNN
        return SEGNN.frag_image_h2([(W, W.shape[1])], None, W.shape[0] // 32, 32, scale)

    # hidden index held by image K slot q = 16 h + 8 m + i of a 32-wide chunk in the fused ConvNext MLP:
    # the register order of the 32x32 MFMA result that becomes GEMM 2's A operand (csrc/ponita.hip
    # po_ffn_kernel)
    FFN_PERM = [(q % 8 & 3) + 16 * ((q // 8) % 2) + 8 * ((q % 8) >> 2) + 4 * (q // 16) for q in range(32)]

    @classmethod
    def _ffn_image(cls, W1, W2):
        """include/nbx.h nbx_ponita_layer.ffn_img_x3: per 32-wide hidden chunk one slab
        [linear_1 rows of the chunk][linear_2 columns of the chunk, K order permuted]."""
        F, C = W1.shape[0], W2.shape[0]
        nj = F // 32
        img1 = cls.lin_image_x3(W1).reshape(nj, -1)                       # [F/32][C/32 blocks]
        perm = torch.tensor([32 * j + q for j in range(nj) for q in cls.FFN_PERM], device=W2.device)
        W2p = W2[:, :F][:, perm].contiguous()
        img2 = cls.lin_image_x3(W2p).reshape(C // 32, nj, -1).transpose(0, 1).reshape(nj, -1)
        return torch.cat([img1, img2], 1).contiguous()

    @staticmethod
    def lin_image_x3(W):
        """[N][Kp] (Kp % 32 == 0, N % 32 == 0) -> int16 bf16x3 image [N/32][Kp/32][3][2][64][8]."""
        from .segnn import SEGNN
        return SEGNN.frag_image_x3([(W, W.shape[1])], None, W.shape[0] // 32, 32)

    def pack_weights(self, device):
        P = self.packed_matrices(device)
        m = self.model
        W = _lib.PonitaWeights()
        W.hidden, W.basis_dim, W.widening = m.hidden_dim, m.basis_dim, m.widening_factor
        W.num_layers, W.num_ori = len(m.interaction_layers), m.num_ori
        for name in ("ori_grid", "basis1_t", "basis1_b", "basis2_t", "basis2_b", "fbasis1_t", "fbasis1_b",
                     "fbasis2_t", "fbasis2_b", "fiber_t", "embed_w"):
            setattr(W, name, P[name].data_ptr())
        W.basis2_img_x3 = P["basis2_img_x3"].data_ptr() if "basis2_img_x3" in P else None
        W.basis_ffn_img_x3 = P["basis_ffn_img_x3"].data_ptr() if "basis_ffn_img_x3" in P else None
        W.basis_ffn_img_h2 = P["basis_ffn_img_h2"].data_ptr() if "basis_ffn_img_h2" in P else None
        W.basis_ffn_h2_s1inv = float(P.get("basis_ffn_h2_s1inv", 1.0))
        W.basis_ffn_h2_s2inv = float(P.get("basis_ffn_h2_s2inv", 1.0))
        for i in range(W.num_layers):
            L = W.layers[i]
            for name, ctype in L._fields_:
                t = P.get(f"layers.{i}.{name}")
                if ctype is _lib.c_f:   # the fp16x2 images' descale factors
                    setattr(L, name, float(t) if t is not None else 1.0)
                else:
                    setattr(L, name, t.data_ptr() if t is not None else None)
        self._packed = (self._param_version(), W, P)
        return W

    def _weights(self, device):
        if self._native_reason:
            raise NotImplementedError(self._native_reason)
        self.model.materialize()
        if self._packed is None or self._packed[0] != self._param_version():
            self.pack_weights(device)
        return self._packed[1]

    def _workspace(self, W, B, N, device):
        n = _lib.c_sz()
        _lib.check(_lib.lib().nbx_ponita_workspace_bytes(W, B, N, n), "ponita workspace")
        if self._ws is None or self._ws.numel() < n.value or self._ws.device != device:
            self._ws = None
            self._ws = torch.empty(n.value, dtype=torch.uint8, device=device)
        return self._ws

    # ------------------------------------------------------------ calibration
    def _needs_callibration(self):
        if not self.training:
            return False
        # the flags are device buffers: their value is cached per (pointer, version), so a steady-state
        # call (e.g. inside a captured training step) makes no host synchronisation
        flags = [L.conv.callibrated for L in self.model.interaction_layers]
        key = tuple((f.data_ptr(), f._version) for f in flags)
        cached = getattr(self, "_calib_cache", None)
        if cached is None or cached[0] != key:
            cached = (key, any(not bool(f) for f in flags))
            self._calib_cache = cached
        return cached[1]

    @torch.no_grad()
    def _callibrate(self, moments, n):
        """FiberBundleConv.callibrate (conv.py:134-140) from per-layer (sum, sum sq)
        of the layer input, x_1 and x_2: unbiased std as torch's Tensor.std()."""
        mom = moments.double().cpu().view(-1, 3, 2)
        std = torch.sqrt((mom[:, :, 1] - mom[:, :, 0] ** 2 / n) / (n - 1))
        for i, L in enumerate(self.model.interaction_layers):
            if bool(L.conv.callibrated):
                continue
            s_in, s_1, s_2 = (float(v) for v in std[i])
            L.conv.kernel.weight.data = L.conv.kernel.weight.data * s_in / s_1
            L.conv.fiber_kernel.weight.data = L.conv.fiber_kernel.weight.data * s_1 / s_2
            L.conv.callibrated = ~L.conv.callibrated

    # ------------------------------------------------------------ forward
    def forward(self, graph):
        """graph: pos, vec / vel, x / mass, edge_index (build_graph_with_knn: fully connected, its kNN
        graphs or any simple graph inside equal-size systems; ``batch`` for the latter)."""
        pos = graph.pos
        device = pos.device
        V = pos.shape[0]
        ei = getattr(graph, "edge_index", None)
        if ei is None:   # this package's own calls: fully connected systems of nbx_system_size nodes
            N = int(graph.nbx_system_size)
            B, fc = V // N, True
        else:
            from .graph import system_layout
            B, N, fc = system_layout(graph, V, ei.shape[1], device)
        f = lambda t: t.detach().to(device=device, dtype=torch.float32).contiguous()
        x = getattr(graph, "x", None)
        if x is None:
            x = graph.mass
        m = f(x.reshape(V))
        vel = graph.vec if getattr(graph, "vec", None) is not None else graph.vel
        p, v = f(pos), f(vel.reshape(V, 3))
        if use_training_path(self):   # train_dispatch.py: autograd on + trainable params
            # training step: native operators under autograd (ponita_train.py).  A model
            # still owing its one-time calibration gets it first from a no-grad forward, as the
            # reference's train.py:49-77 dummy forward does before the first optimiser step.
            if self._native_reason:
                raise NotImplementedError(self._native_reason)
            self.model.materialize()
            if self._needs_callibration():
                with torch.no_grad():
                    self.forward(graph)
            from . import ponita_train
            if ei is None:
                from .graph import fc_edge_index
                ei = fc_edge_index(B, N, device)
            return ponita_train.train_forward(self, p, v, m, ei).to(pos.dtype)
        out = torch.empty(V, 6, device=device, dtype=torch.float32)
        W = self._weights(device)
        ws = self._workspace(W, B, N, device)
        calib = self._needs_callibration()
        mom = torch.zeros(6 * W.num_layers, dtype=torch.float64, device=device) if calib else None
        if fc:
            _lib.check(_lib.lib().nbx_ponita_forward(W, _lib.dev_ptr(p), _lib.dev_ptr(v), _lib.dev_ptr(m), B, N,
                                                     _lib.dev_ptr(out), _lib.dev_ptr(mom) if calib else None,
                                                     _lib.dev_ptr(ws), ws.numel(), _lib.stream_ptr(device)),
                       "nbx_ponita_forward")
        else:
            e = ei.to(device=device, dtype=torch.int64).contiguous()
            _lib.check(_lib.lib().nbx_ponita_forward_graph(
                W, _lib.dev_ptr(p), _lib.dev_ptr(v), _lib.dev_ptr(m), B, N, _lib.dev_ptr(e), e.shape[1],
                _lib.dev_ptr(out), _lib.dev_ptr(mom) if calib else None, _lib.dev_ptr(ws), ws.numel(),
                _lib.stream_ptr(device)), "nbx_ponita_forward_graph")
        self._range_check(W, ws, B, N, device)
        if calib:
            n = V * self.num_ori * self.hidden_dim
            if self.calibration_group is not None:
                import torch.distributed as dist
                if dist.get_world_size(self.calibration_group) > 1:
                    # the (sum, sum sq) moments and the element count over the group's ranks
                    cnt = torch.tensor([float(n)], dtype=torch.float64, device=device)
                    dist.all_reduce(mom, group=self.calibration_group)
                    dist.all_reduce(cnt, group=self.calibration_group)
                    n = int(cnt.item())
            self._callibrate(mom, n)
        return out.to(pos.dtype)

    @torch.no_grad()
    def rollout(self, loc, vel, mass, num_frames: int, absolute: bool = False, num_neighbors=None):
        """Self-feed loop (infer_self_feed.py:131-147,182-194) device-resident:
        loc/vel [B,N,3], mass [B,N,1] -> trajectories [B, T, N, 3] each, frame 0 =
        the initial state.  A model still owing its one-time calibration runs one
        calibrating forward on the initial state first, as the reference's first
        step would.  ``absolute``: pos = pred[:, :3] (targets other than "pos_dt+vel",
        infer_self_feed.py:185-186) instead of pos += pred[:, :3].  ``num_neighbors``: each frame's
        graph is build_graph_with_knn's kNN graph of its positions (None / N-1: fully connected)."""
        flags = _lib.ROLLOUT_ABSOLUTE if absolute else 0
        device = loc.device
        B, N, _ = loc.shape
        knn = num_neighbors is not None and int(num_neighbors) != N - 1
        if knn and int(num_neighbors) >= N:
            raise ValueError("Graph cannot have more neighbors than there are nodes in simulation - 1")

        def run(p_, v_, T, tp_, tv_):
            if knn:
                _lib.check(_lib.lib().nbx_ponita_rollout_knn(
                    W, _lib.dev_ptr(p_), _lib.dev_ptr(v_), _lib.dev_ptr(m), B, N, T, flags, int(num_neighbors),
                    _lib.dev_ptr(tp_), _lib.dev_ptr(tv_), _lib.dev_ptr(ws), ws.numel(), _lib.stream_ptr(device)),
                    "nbx_ponita_rollout_knn")
            else:
                _lib.check(_lib.lib().nbx_ponita_rollout(
                    W, _lib.dev_ptr(p_), _lib.dev_ptr(v_), _lib.dev_ptr(m), B, N, T, flags, _lib.dev_ptr(tp_),
                    _lib.dev_ptr(tv_), _lib.dev_ptr(ws), ws.numel(), _lib.stream_ptr(device)), "nbx_ponita_rollout")
        f = lambda t: t.detach().to(device=device, dtype=torch.float32).contiguous().clone()
        p, v, m = f(loc), f(vel), f(mass.reshape(B * N))
        if self._needs_callibration():
            g = type("G", (), {})()
            g.pos, g.vec, g.x = p.reshape(-1, 3), v.reshape(-1, 1, 3), m.reshape(-1, 1)
            if knn:
                from .graph import build_graph_with_knn
                g.edge_index = build_graph_with_knn(g.pos, B, N, device, int(num_neighbors))
                g.batch = torch.arange(B, device=device).repeat_interleave(N)
            else:
                g.nbx_system_size, g.edge_index = N, None
            first = self.forward(g)
        else:
            first = None
        tp = torch.empty(B, num_frames, N, 3, device=device, dtype=torch.float32)
        tv = torch.empty_like(tp)
        W = self._weights(device)
        ws = self._workspace(W, B, N, device)
        if first is None:
            run(p, v, num_frames, tp, tv)
            self._range_check(W, ws, B, N, device)
            return tp, tv
        # frame 1 came from the calibrating forward; the rest from the calibrated weights
        tp[:, 0], tv[:, 0] = p, v
        if num_frames == 1:
            return tp, tv
        p = first[:, :3].reshape(B, N, 3).contiguous() if absolute else p + first[:, :3].reshape(B, N, 3)
        v = first[:, 3:].reshape(B, N, 3).contiguous()
        rp = torch.empty(B, num_frames - 1, N, 3, device=device, dtype=torch.float32)
        rv = torch.empty_like(rp)
        run(p, v, num_frames - 1, rp, rv)
        self._range_check(W, ws, B, N, device)
        tp[:, 1:], tv[:, 1:] = rp, rv
        return tp, tv

    def _range_check(self, W, ws, B, N, device):
        """fp16x2 range guard (include/nbx.h nbx_ponita_range_check): NbxError instead of non-finite results
        when a GEMM operand leaves the fp16 range of the split path; one stream synchronisation per call,
        skipped while a HIP graph is captured and when ``range_check`` is False."""
        if getattr(self, "range_check", True) and not torch.cuda.is_current_stream_capturing():
            _lib.check(_lib.lib().nbx_ponita_range_check(W, _lib.dev_ptr(ws), ws.numel(), B, N,
                                                         _lib.stream_ptr(device)), "ponita")
