"""SEGNN — drop-in for models/segnn/segnn.py::SEGNN with a fused HIP forward.

Module tree, parameter names, shapes, init ranges and state_dict keys follow the
reference (segnn.py:17-304, o3_building_blocks.py:10-203, e3nn BatchNorm), so a
reference checkpoint loads into this class.  ``forward(graph)`` runs O3Transform +
catch_isolated_nodes + the SEGNN forward (fp32) inside libnbx (csrc/segnn.hip);
``rollout`` runs the whole self-feed loop device-resident.

Native scope (anything else raises NotImplementedError): task="node", norm="batch",
lmax_h = lmax_attr = 1, input 2x1o+1x0e, output 2x1o, additional message
irreps 2x0e, fully-connected systems of equal size.
"""
from __future__ import annotations

import math
import warnings
import weakref

import torch
import torch.nn as nn

from . import _lib
from .train_dispatch import use_training_path
from .o3 import FullyConnectedTensorProduct, Irreps, weight_balanced_irreps

SH_C0 = 1.0 / math.sqrt(4.0 * math.pi)
SH_C1 = math.sqrt(3.0 / (4.0 * math.pi))
INV_SQRT3 = 1.0 / math.sqrt(3.0)


def _destroy_comm(comm):
    """Release a library RCCL communicator (after the device has drained the work enqueued on it)."""
    try:
        torch.cuda.synchronize()
    finally:
        _lib.check(_lib.lib().nbx_comm_destroy(comm), "nbx_comm_destroy")


class O3TensorProduct(nn.Module):
    """o3_building_blocks.py:10-167: e3nn FCTP + sqrt(fan_in) rescale + 0e biases.
    Init: e3nn randn, then U(-1/sqrt(fan_in), +) per instruction block and bias."""

    def __init__(self, irreps_in1, irreps_out, irreps_in2=None, tp_rescale=True):
        super().__init__()
        self.irreps_in1 = Irreps(irreps_in1)
        self.irreps_out = Irreps(irreps_out)
        self.irreps_in2_provided = irreps_in2 is not None
        self.irreps_in2 = Irreps(irreps_in2) if irreps_in2 is not None else Irreps("1x0e")
        self.tp_rescale = tp_rescale
        self.tp = FullyConnectedTensorProduct(self.irreps_in1, self.irreps_in2, self.irreps_out)
        fan_in = {}
        for ins in self.tp.instructions:
            fan_in[ins.i_out] = fan_in.get(ins.i_out, 0) + ins.shape[0] * ins.shape[1]
        self.fan_in = fan_in
        bias_slots = [io for io, (m, ir) in enumerate(self.irreps_out) if ir.l == 0]
        with torch.no_grad():
            for w, ins in zip(self.tp.weight_views(), self.tp.instructions):
                k = 1.0 / math.sqrt(fan_in[ins.i_out]) if tp_rescale else 1.0
                w.uniform_(-k, k)
            biases = []
            for io in bias_slots:
                k = 1.0 / math.sqrt(fan_in[io])
                biases.append(torch.zeros(self.irreps_out[io][0]).uniform_(-k, k))
        self.biases = nn.Parameter(torch.cat(biases)) if biases else None

    def forward(self, *a):  # pragma: no cover
        raise NotImplementedError("O3 tensor products run fused inside the SEGNN HIP kernels")


class O3TensorProductSwishGate(O3TensorProduct):
    """o3_building_blocks.py:170-203: TP to (scalars + gates + gated).simplify()."""

    def __init__(self, irreps_in1, irreps_out, irreps_in2=None):
        irreps_out = Irreps(irreps_out)
        scalars = Irreps([irreps_out[0]])
        gates = Irreps(f"{irreps_out.num_irreps - scalars.num_irreps}x0e")
        gated = Irreps(irreps_out[1:])
        super().__init__(irreps_in1, (scalars + gates + gated).simplify(), irreps_in2)
        self.irreps_gated = gated


class BatchNorm(nn.Module):
    """e3nn.nn.BatchNorm parameter/buffer layout (affine, reduce="mean",
    normalization="component", eps=1e-5, momentum=0.1)."""

    def __init__(self, irreps, eps=1e-5, momentum=0.1):
        super().__init__()
        self.irreps = Irreps(irreps)
        self.eps, self.momentum = eps, momentum
        n_scalar = sum(m for m, ir in self.irreps if ir.l == 0 and ir.p == 1)
        self.weight = nn.Parameter(torch.ones(self.irreps.num_irreps))
        self.bias = nn.Parameter(torch.zeros(n_scalar))
        self.register_buffer("running_mean", torch.zeros(n_scalar))
        self.register_buffer("running_var", torch.ones(self.irreps.num_irreps))


class _TrainPackFn(torch.autograd.Function):
    """SEGNN._train_layout's gather: (layout, *flat tensor-product weights) -> the operand tensors."""

    @staticmethod
    def forward(ctx, L, *weights):
        flat = torch.cat([w.reshape(-1).to(torch.float32) for w in weights] +
                         [torch.zeros(1, device=L["src"].device, dtype=torch.float32)])
        buf = flat.index_select(0, L["src"]).mul_(L["scale"])
        ctx.L = L
        ctx.meta = [(w.dtype, w.shape) for w in weights]
        return tuple(buf[o:o + math.prod(sh)].view(sh) for o, sh in L["slots"].values())

    @staticmethod
    def backward(ctx, *grads):
        L = ctx.L
        parts = [g.reshape(-1) if g is not None else torch.zeros(math.prod(sh), device=L["src"].device)
                 for g, (o, sh) in zip(grads, L["slots"].values())]
        dbuf = torch.cat(parts).mul_(L["scale"])
        dflat = torch.zeros(L["total"], device=dbuf.device, dtype=torch.float32)
        dflat.index_put_((L["live_src"],), dbuf.index_select(0, L["live_pos"]))   # unique targets
        return (None,) + tuple(d.view(sh).to(dt) for d, (dt, sh) in zip(dflat.split(L["sizes"]), ctx.meta))


class SEGNNLayer(nn.Module):
    """segnn.py:192-304 (PyG MessagePassing, aggr="add", node_dim=-2)."""

    def __init__(self, input_irreps, hidden_irreps, output_irreps, edge_attr_irreps, node_attr_irreps,
                 norm=None, additional_message_irreps=None):
        super().__init__()
        self.hidden_irreps = hidden_irreps
        msg_in = (input_irreps + input_irreps + additional_message_irreps).simplify()
        upd_in = (input_irreps + hidden_irreps).simplify()
        self.message_layer_1 = O3TensorProductSwishGate(msg_in, hidden_irreps, edge_attr_irreps)
        self.message_layer_2 = O3TensorProductSwishGate(hidden_irreps, hidden_irreps, edge_attr_irreps)
        self.update_layer_1 = O3TensorProductSwishGate(upd_in, hidden_irreps, node_attr_irreps)
        self.update_layer_2 = O3TensorProduct(hidden_irreps, hidden_irreps, node_attr_irreps)
        self.norm = norm
        self.feature_norm = self.message_norm = None
        if norm == "batch":
            self.feature_norm = BatchNorm(hidden_irreps)
            self.message_norm = BatchNorm(hidden_irreps)
        elif norm is not None:
            raise NotImplementedError(f"SEGNN norm={norm!r} is outside the native path")


class SEGNN(nn.Module):
    """Steerable E(3) equivariant message passing network (segnn.py:14-189)."""

    def __init__(self, input_irreps="2x1o + 1x0e", hidden_features=64, lmax_h=1, lmax_attr=1, num_layers=4,
                 output_irreps="2x1o", norm="batch", pool="avg", task="node", additional_message_irreps="2x0e",
                 training_args=None, deterministic=False):
        super().__init__()
        if task != "node" or lmax_h != 1 or lmax_attr != 1 or norm != "batch":
            raise NotImplementedError("native SEGNN supports task='node', norm='batch', lmax_h = lmax_attr = 1")
        self.hidden_features, self.lmax_h, self.lmax_attr, self.num_layers = hidden_features, lmax_h, lmax_attr, num_layers
        self.node_attr_irreps = Irreps.spherical_harmonics(lmax_attr)
        hidden_irreps = weight_balanced_irreps(hidden_features, self.node_attr_irreps, lmax_h)
        self.edge_attr_irreps = Irreps.spherical_harmonics(lmax_attr)
        self.hidden_irreps, self.task, self.norm, self.pool = hidden_irreps, task, norm, pool
        self.additional_message_irreps = Irreps(additional_message_irreps)
        self.training_args = training_args
        input_irreps, output_irreps = Irreps(input_irreps), Irreps(output_irreps)
        if str(input_irreps) != "2x1o+1x0e" or str(output_irreps) != "2x1o" or \
                str(self.additional_message_irreps) != "2x0e":
            raise NotImplementedError("native SEGNN expects 2x1o+1x0e -> 2x1o with 2x0e message features")
        self.embedding_layer = O3TensorProduct(input_irreps, hidden_irreps, self.node_attr_irreps)
        self.layers = nn.ModuleList([
            SEGNNLayer(hidden_irreps, hidden_irreps, hidden_irreps, self.edge_attr_irreps, self.node_attr_irreps,
                       norm=norm, additional_message_irreps=self.additional_message_irreps)
            for _ in range(num_layers)])
        self.pre_pool1 = O3TensorProductSwishGate(hidden_irreps, hidden_irreps, self.node_attr_irreps)
        self.pre_pool2 = O3TensorProduct(hidden_irreps, output_irreps, self.node_attr_irreps)
        self.mul = hidden_irreps[0][0]
        if str(hidden_irreps) != f"{self.mul}x0e+{self.mul}x1o" or self.mul % 4:
            raise NotImplementedError(f"hidden irreps {hidden_irreps} outside the native path (mul % 4 == 0)")
        self._packed = None
        self._ws = None
        self._tlayout = None         # training operand layout (_train_layout)
        self._warned_dtype = False
        self._bn_group = None        # SyncBN process group (enable_sync_batchnorm)
        self._bn_global_batch = None
        self._bn_comm_fin = None
        self._bn_hook = None
        self._bn_comm = None         # RCCL communicator the library all-reduces on (nbx_comm_init)
        # deterministic=True: train-mode BatchNorm sums reduced in a fixed order instead of fp64
        # atomics, so repeated train-mode forwards / rollouts are bit-identical (include/nbx.h)
        self.deterministic = bool(deterministic)
        # BatchNorm statistics of the native forward / rollout (SURVEY §8(e) bn_mode): None follows
        # self.training like the reference module (train() -> batch statistics, the reference's
        # rollout semantics, infer_self_feed.py never calls eval()); "batch" / "running" force
        # batch statistics (running stats updated) / the running statistics
        self.bn_mode = None
        # fp16x2 range guard after every native forward / rollout (include/nbx.h nbx_segnn_range_check):
        # NbxError instead of non-finite results when an operand leaves the fp16 range of the split path
        self.range_check = True

    # ------------------------------------------------------------ reference API
    def get_model_size(self):
        return self.hidden_features

    def get_serializable_attributes(self):
        return {
            "hidden_features": self.hidden_features, "lmax_h": self.lmax_h, "lmax_attr": self.lmax_attr,
            "node_attr_irreps": str(self.node_attr_irreps), "num_layers": self.num_layers,
            "input_irreps": str(self.embedding_layer.irreps_in1), "hidden_irreps": str(self.hidden_irreps),
            "output_irreps": str(self.pre_pool2.irreps_out), "edge_attr_irreps": str(self.edge_attr_irreps),
            "norm": self.norm, "pool": None, "task": self.task,
            "additional_message_irreps": str(self.additional_message_irreps),
            "training_args": self.training_args, "num_params": sum(p.numel() for p in self.parameters()),
        }

    # ------------------------------------------------------------ weight packing
    def _param_version(self):
        return tuple((p.data_ptr(), p._version) for p in self.parameters()) + \
            tuple((b.data_ptr(), b.dtype) for b in self.buffers())

    def packed_matrices(self, device="cpu", dtype=torch.float32):
        """The e3nn parameters re-packed into the fp32 GEMM operands of include/nbx.h
        (M = mul, c0/c1 = SH prefactors, s3 = 1/sqrt 3; derivation in DESIGN.md §SEGNN).
        Matrices named *_t are [N_out][K_in]."""
        M = self.mul
        f32 = dict(device=device, dtype=dtype)

        def views(tpmod):
            return [w.detach().to(**f32)[:, 0, :] for w in tpmod.tp.weight_views()]   # [mul1, mul_out]

        def T(x):
            return x.t().contiguous()

        def vec(x):
            return x.detach().to(**f32).contiguous()

        z = torch.zeros(M, M, **f32)
        P = {}
        Wa, Wb, Wc, Wd = views(self.embedding_layer)
        P["emb"] = vec(torch.stack([Wa[0], Wa[1], Wb[0] * INV_SQRT3, Wb[1] * INV_SQRT3, Wc[0], Wd[0]]))
        P["emb_bias"] = vec(self.embedding_layer.biases)
        for li, layer in enumerate(self.layers):
            p = f"layers.{li}."
            WA0, WA1, WB0, WB1, WC0, WC1, WD0, WD1, WE0, WE1 = views(layer.message_layer_1)
            P[p + "node_pre_s_t"] = T(torch.cat([SH_C0 * WA0, SH_C1 * WA1, SH_C0 * WC0, SH_C1 * WC1], 1))
            P[p + "node_pre_v_t"] = T(torch.cat([SH_C1 * INV_SQRT3 * WB1, SH_C0 * WB0,
                                                 SH_C1 * INV_SQRT3 * WD1, SH_C0 * WD0], 1))
            P[p + "msg1_amf"] = vec(torch.cat([SH_C0 * WE0, SH_C1 * WE1], 1))
            P[p + "msg1_bias"] = vec(layer.message_layer_1.biases)
            W1, W2, W3, W4 = views(layer.message_layer_2)
            P[p + "msg2_s_t"] = T(torch.cat([torch.cat([SH_C0 * W1, SH_C1 * INV_SQRT3 * W4], 0),
                                             torch.cat([SH_C1 * W2, z], 0)], 1))
            P[p + "msg2_v_t"] = T(SH_C0 * W3)
            P[p + "msg2_bias"] = vec(layer.message_layer_2.biases)
            Xs0, Xs1, Xv0, Xv1, As0, As1, Av0, Av1 = views(layer.update_layer_1)
            P[p + "upd1_s_t"] = T(torch.cat([torch.cat([Xs0, As0, INV_SQRT3 * Xv1, INV_SQRT3 * Av1], 0),
                                             torch.cat([Xs1, As1, z, z], 0)], 1))
            P[p + "upd1_v_t"] = T(torch.cat([Xv0, Av0], 0))
            P[p + "upd1_bias"] = vec(layer.update_layer_1.biases)
            U1, U2, U3, U4 = views(layer.update_layer_2)
            P[p + "upd2_s_t"] = T(torch.cat([torch.cat([U1, INV_SQRT3 * U4], 0), torch.cat([U2, z], 0)], 1))
            P[p + "upd2_v_t"] = T(U3)
            P[p + "upd2_bias"] = vec(layer.update_layer_2.biases)
            for name, bn in (("msg", layer.message_norm), ("feat", layer.feature_norm)):
                P[p + f"{name}_bn_weight"] = vec(bn.weight)
                P[p + f"{name}_bn_bias"] = vec(bn.bias)
        P1, P2, P3, P4 = views(self.pre_pool1)
        P["pp1_s_t"] = T(torch.cat([torch.cat([P1, INV_SQRT3 * P4], 0), torch.cat([P2, z], 0)], 1))
        P["pp1_v_t"] = T(P3)
        P["pp1_bias"] = vec(self.pre_pool1.biases)
        Ws, Wv = views(self.pre_pool2)
        P["pp2"] = vec(torch.stack([Ws[:, 0], Ws[:, 1], Wv[:, 0], Wv[:, 1]]))
        return P

    def train_matrices(self, device, weights=None, dtype=torch.float32):
        """The operands of the training step's canonical tensor products (include/nbx.h "SEGNN
        training step"; segnn_train.py), built from the e3nn parameters with differentiable torch
        ops: ``<tp>_s`` = Ws [NSc + Nt][Ks + Kv], ``<tp>_v`` = Wv [Nt][Kv], ``<tp>_bias``.  Same
        constants as packed_matrices; message_layer_1 unfactored, its input being
        [x_i s | x_j s | amf | x_i v . rhat | x_j v . rhat] and [x_i v | x_j v] per edge.
        ``weights``: {id(O3TensorProduct): flat weight} in place of the modules' own (the layout
        trace of :meth:`train_operands`)."""
        M = self.mul
        f32 = dict(device=device, dtype=dtype)

        def views(tpmod):
            w = None if weights is None else weights[id(tpmod)]
            return [v.to(**f32)[:, 0, :] for v in tpmod.tp.weight_views(w)]   # [mul1, mul_out]

        def T(x):
            return x.t().contiguous()

        z = lambda r, c: torch.zeros(r, c, **f32)
        P = {}
        Wa, Wb, Wc, Wd = views(self.embedding_layer)          # S_in = [|v| | pos_c . na | vel . na]
        P["emb_s"] = T(torch.cat([torch.stack([Wc[0], Wb[0] * INV_SQRT3, Wb[1] * INV_SQRT3]),
                                  torch.stack([Wd[0], Wd[0] * 0, Wd[0] * 0])], 1))
        P["emb_v"] = T(Wa)
        P["emb_bias"] = self.embedding_layer.biases.to(**f32)
        for li, layer in enumerate(self.layers):
            p = f"layers.{li}."
            WA0, WA1, WB0, WB1, WC0, WC1, WD0, WD1, WE0, WE1 = views(layer.message_layer_1)
            s_blk = torch.cat([SH_C0 * WA0, SH_C0 * WC0, SH_C0 * WE0, SH_C1 * INV_SQRT3 * WB1, SH_C1 * INV_SQRT3 * WD1])
            t_blk = torch.cat([SH_C1 * WA1, SH_C1 * WC1, SH_C1 * WE1, z(2 * M, M)])
            P[p + "msg1_s"] = T(torch.cat([s_blk, t_blk], 1))
            P[p + "msg1_v"] = T(torch.cat([SH_C0 * WB0, SH_C0 * WD0]))
            P[p + "msg1_bias"] = layer.message_layer_1.biases.to(**f32)
            W1, W2, W3, W4 = views(layer.message_layer_2)
            P[p + "msg2_s"] = T(torch.cat([torch.cat([SH_C0 * W1, SH_C1 * INV_SQRT3 * W4]),
                                           torch.cat([SH_C1 * W2, z(M, M)])], 1))
            P[p + "msg2_v"] = T(SH_C0 * W3)
            P[p + "msg2_bias"] = layer.message_layer_2.biases.to(**f32)
            Xs0, Xs1, Xv0, Xv1, As0, As1, Av0, Av1 = views(layer.update_layer_1)
            P[p + "upd1_s"] = T(torch.cat([torch.cat([Xs0, As0, INV_SQRT3 * Xv1, INV_SQRT3 * Av1]),
                                           torch.cat([Xs1, As1, z(2 * M, M)])], 1))
            P[p + "upd1_v"] = T(torch.cat([Xv0, Av0]))
            P[p + "upd1_bias"] = layer.update_layer_1.biases.to(**f32)
            U1, U2, U3, U4 = views(layer.update_layer_2)
            P[p + "upd2_s"] = T(torch.cat([torch.cat([U1, INV_SQRT3 * U4]), torch.cat([U2, z(M, M)])], 1))
            P[p + "upd2_v"] = T(U3)
            P[p + "upd2_bias"] = layer.update_layer_2.biases.to(**f32)
        P1, P2, P3, P4 = views(self.pre_pool1)
        P["pp1_s"] = T(torch.cat([torch.cat([P1, INV_SQRT3 * P4]), torch.cat([P2, z(M, M)])], 1))
        P["pp1_v"] = T(P3)
        P["pp1_bias"] = self.pre_pool1.biases.to(**f32)
        Ws, Wv = views(self.pre_pool2)
        P["pp2_s"] = T(torch.cat([Ws, z(M, 2)]))
        P["pp2_v"] = T(Wv)
        return P

    def _train_layout(self, device):
        """The map from the concatenated tensor-product weights to every operand of
        :meth:`train_matrices`, traced once (the layout depends on the module structure only):
        operand element i = scale[i] * flat[src[i]], or 0 (src = the appended zero slot).  Every
        weight element feeds at most one operand element, so the backward is a scatter."""
        if self._tlayout is not None and self._tlayout["device"] == device:
            return self._tlayout
        tps = [m for m in self.modules() if isinstance(m, O3TensorProduct)]
        sizes = [m.tp.weight.numel() for m in tps]
        total = sum(sizes)
        ids, ones, perm_ids, off = {}, {}, {}, 0
        # a third trace with the element ids permuted at random: an operand element c w_a + c w_b with
        # equal constants would pass the id / ones traces as w_{(a+b)/2}, but not this one
        perm = torch.randperm(total, generator=torch.Generator().manual_seed(1234)).to(torch.float64) + 1
        for m, n in zip(tps, sizes):
            ids[id(m)] = torch.arange(off + 1, off + n + 1, dtype=torch.float64)   # 1-based: 0 = no source
            ones[id(m)] = torch.ones(n, dtype=torch.float64)
            perm_ids[id(m)] = perm[off:off + n]
            off += n
        cpu = torch.device("cpu")
        with torch.no_grad():
            Pi = self.train_matrices(cpu, ids, torch.float64)
            Po = self.train_matrices(cpu, ones, torch.float64)
            Pp = self.train_matrices(cpu, perm_ids, torch.float64)
        keys = [k for k in Pi if not k.endswith("_bias")]
        src, scale, slots = [], [], {}
        pos = 0
        for k in keys:
            vi, vo = Pi[k].reshape(-1), Po[k].reshape(-1)
            live = vo != 0
            idx = torch.where(live, torch.round(vi / torch.where(live, vo, torch.ones_like(vo))), torch.zeros_like(vi))
            if not torch.equal(idx * vo, torch.where(live, vi, torch.zeros_like(vi))) and \
                    not torch.allclose(idx * vo, vi, rtol=1e-12, atol=0):
                raise RuntimeError(f"SEGNN training operand {k} is not a scaled copy of the weights")
            vp = Pp[k].reshape(-1)
            want = torch.where(live, perm[(idx - 1).clamp(min=0).long()] * vo, torch.zeros_like(vo))
            if not torch.allclose(vp, want, rtol=1e-12, atol=0):
                raise RuntimeError(f"SEGNN training operand {k} mixes several weights")
            src.append(torch.where(live, idx - 1, torch.full_like(idx, total)).long())
            scale.append(torch.where(live, vo, torch.zeros_like(vo)))
            slots[k] = (pos, tuple(Pi[k].shape))
            pos += vi.numel()
        src, scale = torch.cat(src), torch.cat(scale)
        live = src < total
        if torch.unique(src[live]).numel() != int(live.sum()):
            raise RuntimeError("SEGNN training operands: a weight element feeds two operand elements")
        self._tlayout = {"device": device, "tps": tps, "sizes": sizes, "slots": slots,
                         "src": src.to(device), "scale": scale.to(device=device, dtype=torch.float32),
                         "live_pos": torch.nonzero(live).reshape(-1).to(device),
                         "live_src": src[live].to(device), "total": total}
        return self._tlayout

    def train_operands(self, device):
        """:meth:`train_matrices` as one gather: the concatenated tensor-product weights -> every
        operand (scale x weight), and in the backward one scatter of the operand gradients back
        (_TrainPackFn).  Equal to train_matrices element for element (a product by the same
        constant); a few launches instead of hundreds of small differentiable torch ops."""
        L = self._train_layout(device)
        outs = _TrainPackFn.apply(L, *[m.tp.weight for m in L["tps"]])
        P = dict(zip(L["slots"], outs))
        f32 = dict(device=device, dtype=torch.float32)
        P["emb_bias"] = self.embedding_layer.biases.to(**f32)
        for li, layer in enumerate(self.layers):
            p = f"layers.{li}."
            for name, mod in (("msg1", layer.message_layer_1), ("msg2", layer.message_layer_2),
                              ("upd1", layer.update_layer_1), ("upd2", layer.update_layer_2)):
                P[p + name + "_bias"] = mod.biases.to(**f32)
        P["pp1_bias"] = self.pre_pool1.biases.to(**f32)
        return P

    # ------------------------------------------------------------ LDS images (include/nbx.h)
    @staticmethod
    def frag_image(subs, vec, cw: int, chunks: int) -> torch.Tensor:
        """MFMA-fragment-ordered weight image of one TP (include/nbx.h "TP operand
        images"): `subs` = [(W_j [rows][>=K_j], K_j)] scalar sub-tiles, `vec` = (W_v, K_v) or
        None; row c of every matrix is output channel c of that part.  Returns
        [chunks][F] fp32, chunk = `cw` channels of every part, zero-filled past K and
        past the real rows."""
        blocks = []
        for W, K in list(subs) + ([vec] if vec is not None else []):
            kc = (K + 31) // 32
            X = torch.zeros(chunks * cw, kc * 32, dtype=W.dtype, device=W.device)
            n = min(W.shape[0], chunks * cw)
            X[:n, :K] = W[:n, :K]
            if cw == 16:   # [c][16][kc][qd 4][half 2][e 4] -> [c][kc][half][qd][16][e]
                X = X.reshape(chunks, 16, kc, 4, 2, 4).permute(0, 2, 4, 3, 1, 5)
            else:          # [c][32][kc][h 2][q 4][e 4] -> [c][kc][q][h][32][e]
                X = X.reshape(chunks, 32, kc, 2, 4, 4).permute(0, 2, 4, 3, 1, 5)
            blocks.append(X.reshape(chunks, -1))
        return torch.cat(blocks, 1).contiguous()

    @staticmethod
    def split_bf16x3(W: torch.Tensor):
        """W = hi + mid + lo with each part rounded to bf16 (residual <= 2^-27 |W|): the
        operands of the split-precision MFMA path (include/nbx.h "bf16x3 images")."""
        W = W.float()
        hi = W.to(torch.bfloat16)
        r = W - hi.float()
        mid = r.to(torch.bfloat16)
        lo = (r - mid.float()).to(torch.bfloat16)
        return hi, mid, lo

    @staticmethod
    def frag_image_x3(subs, vec, chunks: int, cw: int = 32) -> torch.Tensor:
        """bf16x3 image (include/nbx.h "bf16x3 images"), per sub-tile and 32-deep K chunk kc:
          cw = 32 (v_mfma_f32_32x32x16_bf16): block [part p 3][m 2][lane 64][j 8] = part p of
                  W[c = 32 chunk + (lane & 31)][k = 32 kc + 16 (lane >> 5) + 8 m + j];
          cw = 16 (v_mfma_f32_16x16x32_bf16): block [part p 3][lane 64][j 8] = part p of
                  W[c = 16 chunk + (lane & 15)][k = 32 kc + 8 (lane >> 4) + j];
        zero past K / rows.  Returned as int16 bit patterns [chunks][F16]."""
        blocks = []
        for W, K in list(subs) + ([vec] if vec is not None else []):
            kc = (K + 31) // 32
            X = torch.zeros(chunks * cw, kc * 32, dtype=torch.float32, device=W.device)
            n = min(W.shape[0], chunks * cw)
            X[:n, :K] = W[:n, :K].float()
            parts = torch.stack([t.float() for t in SEGNN.split_bf16x3(X)])      # [3][rows][kc*32]
            if cw == 32:
                # [p][c][r 32][kc][h 2][m 2][j 8] -> [c][kc][p][m][h][r][j]
                Y = parts.reshape(3, chunks, 32, kc, 2, 2, 8).permute(1, 3, 0, 5, 4, 2, 6)
            else:
                # [p][c][r 16][kc][qd 4][j 8] -> [c][kc][p][qd][r][j]
                Y = parts.reshape(3, chunks, 16, kc, 4, 8).permute(1, 3, 0, 4, 2, 5)
            blocks.append(Y.reshape(chunks, -1))
        img = torch.cat(blocks, 1).contiguous().to(torch.bfloat16)
        return img.view(torch.int16)

    @staticmethod
    def h2_scale(*mats) -> float:
        """The power of two s with max |W s| in [2^9, 2^10) over the given matrices (1 if all zero):
        the fp16x2 images' weight scale (include/nbx.h "fp16x2 images")."""
        m = max(float(W.abs().max()) if W.numel() else 0.0 for W in mats)
        if m == 0.0 or not math.isfinite(m):
            return 1.0
        return 2.0 ** (9 - math.floor(math.log2(m)))

    @staticmethod
    def frag_image_h2(subs, vec, chunks: int, cw: int, scale: float) -> torch.Tensor:
        """fp16x2 image (include/nbx.h "fp16x2 images"): W s = hi + lo, hi = fp16(W s) (RNE),
        lo = fp16(W s - hi); per sub-tile and 32-deep K chunk kc the bf16x3 block layout of
        frag_image_x3 with two fp16 parts:
          cw = 32: block [part p 2][m 2][lane 64][j 8],  cw = 16: block [part p 2][lane 64][j 8].
        Returned as int16 bit patterns [chunks][F16]."""
        blocks = []
        for W, K in list(subs) + ([vec] if vec is not None else []):
            kc = (K + 31) // 32
            X = torch.zeros(chunks * cw, kc * 32, dtype=torch.float64, device=W.device)
            n = min(W.shape[0], chunks * cw)
            X[:n, :K] = W[:n, :K].double() * scale
            X = X.float()                                   # exact: scale is a power of two
            hi = X.half()
            lo = (X - hi.float()).half()                    # the residual is exact in fp32
            parts = torch.stack([hi.float(), lo.float()])   # [2][rows][kc*32]
            if cw == 32:
                Y = parts.reshape(2, chunks, 32, kc, 2, 2, 8).permute(1, 3, 0, 5, 4, 2, 6)
            else:
                Y = parts.reshape(2, chunks, 16, kc, 4, 8).permute(1, 3, 0, 4, 2, 5)
            blocks.append(Y.reshape(chunks, -1))
        img = torch.cat(blocks, 1).contiguous().half()
        return img.view(torch.int16)

    @staticmethod
    def tp_images(P: dict, mul: int) -> dict:
        """packed_matrices -> the device images the kernels stage (msg2: 32-channel
        chunks for the 32x32 message kernel; every other TP: 16-channel chunks, the
        chunk count padded to a multiple of 4 so any channel-group size <= 4 divides it;
        node_pre: 6 parts [P_dst s|gate|t, P_src s|gate|t] per 16-channel chunk)."""
        M = mul
        c16 = -(-M // 16)
        c16 = -(-c16 // 4) * 4
        c32 = -(-M // 32)
        img = SEGNN.frag_image
        out = {}
        for key in list(P):
            pre, base = (key.rsplit(".", 1) + [""])[:2] if "." in key else ("", key)
            pre = pre + "." if pre else ""
            if base in ("node_pre_s_t", "node_pre_v_t"):
                B = P[key]                                    # [6M][M]: 6 parts of M output columns
                subs = [(B[j * M:(j + 1) * M], M) for j in range(6)]
                out[pre + base[:-2] + "_img"] = img(subs, None, 16, c16)
                out[pre + base[:-2] + "_img_x3"] = SEGNN.frag_image_x3(subs, None, c16, 16)
                # one scale for both node_pre images (one kernel, one descale)
                sc = SEGNN.h2_scale(P[pre + "node_pre_s_t"], P[pre + "node_pre_v_t"])
                out[pre + base[:-2] + "_img_h2"] = SEGNN.frag_image_h2(subs, None, c16, 16, sc)
                out[pre + "node_pre_h2_descale"] = 1.0 / sc
            elif base in ("msg2_s_t", "upd1_s_t", "upd2_s_t", "pp1_s_t"):
                stem = base[:-4]
                S, V = P[key], P[pre + stem + "_v_t"]
                K = S.shape[1]
                parts = S.shape[0] // M
                # the last part (t, 0e -> 1o path) only contracts the first half of K
                Ks = [K] * (parts - 1) + [K // 2]
                subs = [(S[j * M:(j + 1) * M], Ks[j]) for j in range(parts)]
                sc = SEGNN.h2_scale(S, V)
                out[pre + stem + "_h2_descale"] = 1.0 / sc
                if stem == "msg2":
                    out[pre + stem + "_img"] = img(subs, (V, V.shape[1]), 32, c32)
                    out[pre + stem + "_img_x3"] = SEGNN.frag_image_x3(subs, (V, V.shape[1]), c32)
                    out[pre + stem + "_img_h2"] = SEGNN.frag_image_h2(subs, (V, V.shape[1]), c32, 32, sc)
                else:
                    out[pre + stem + "_img"] = img(subs, (V, V.shape[1]), 16, c16)
                    out[pre + stem + "_img_h2"] = SEGNN.frag_image_h2(subs, (V, V.shape[1]), c16, 16, sc)
                    if stem == "upd1":
                        out[pre + stem + "_img_x3"] = SEGNN.frag_image_x3(subs, (V, V.shape[1]), c16, 16)
            elif base.endswith("_v_t"):
                continue
            else:
                out[key] = P[key]
        return out

    def _bn_buffers(self):
        for layer in self.layers:
            for bn in (layer.message_norm, layer.feature_norm):
                yield bn.running_mean
                yield bn.running_var

    def pack_weights(self, device):
        """Build the nbx_segnn_weights struct (device pointers) from packed_matrices.

        The kernels update the BatchNorm running statistics in place in fp32.  When the
        module's buffers are fp32 device tensors the struct points straight at them; after
        ``model.double()`` (the reference's default precision_mode, infer_self_feed.py:45-48)
        it points at fp32 device shadows that ``_bn_sync_in`` / ``_bn_sync_out`` copy from /
        back into the fp64 buffers around every native call."""
        P = self.tp_images(self.packed_matrices(device), self.mul)
        W = _lib.SegnnWeights()
        W.mul, W.num_layers, W.bn_eps, W.bn_momentum = self.mul, self.num_layers, 1e-5, 0.1
        for k in ("emb", "emb_bias", "pp1_img", "pp1_bias", "pp2", "pp1_img_h2"):
            setattr(W, k, P[k].data_ptr())
        W.pp1_h2_descale = P["pp1_h2_descale"]
        shadows = []
        for li, layer in enumerate(self.layers):
            L = W.layers[li]
            for name, _ in L._fields_:
                key = f"layers.{li}.{name}"
                if key in P:
                    setattr(L, name, P[key] if isinstance(P[key], float) else P[key].data_ptr())
            for name, bn in (("msg", layer.message_norm), ("feat", layer.feature_norm)):
                for stat in ("running_mean", "running_var"):
                    buf = getattr(bn, stat)
                    if not buf.is_cuda:
                        raise _lib.NbxError("BatchNorm running stats must live on the HIP device")
                    if buf.dtype == torch.float32 and buf.is_contiguous():
                        setattr(L, f"{name}_bn_{stat}", buf.data_ptr())   # updated in place
                    else:
                        sh = torch.empty(buf.shape, dtype=torch.float32, device=buf.device)
                        shadows.append((buf, sh))
                        setattr(L, f"{name}_bn_{stat}", sh.data_ptr())
        self._packed = (self._param_version(), W, P, shadows)
        return W

    def _bn_batch(self):
        """True when the native path uses (and updates) batch statistics (bn_mode, else self.training)."""
        if self.bn_mode not in (None, "batch", "running"):
            raise ValueError(f"bn_mode must be None, 'batch' or 'running' (got {self.bn_mode!r})")
        return self.training if self.bn_mode is None else self.bn_mode == "batch"

    def invalidate_weights(self):
        """Drop the packed inference operands (rebuilt at the next native call).  Needed after
        parameter updates that do not bump the version counters, e.g. replays of a captured training
        step (HIP graph) whose optimizer writes the parameters in place on the device."""
        self._packed = None
        return self

    def _weights(self, device):
        if self._packed is None or self._packed[0] != self._param_version():
            self.pack_weights(device)
        W = self._packed[1]
        W.training = 1 if self._bn_batch() else 0
        W.deterministic = 1 if self.deterministic else 0
        return W

    # ------------------------------------------------------------ SyncBN (multi-GPU)
    def enable_sync_batchnorm(self, group=None, use_rccl=None, global_batch=None):
        """Train-mode BatchNorm over the union of every rank's batch (the reference's
        single-process statistics, segnn.py:233-235,257-261,282-283, when the batch is sharded
        over ranks): after each producing kernel the [3][mul] fp64 sums of that BatchNorm are
        all-reduced over the ranks on the launch stream and normalised by the global counts.
        12 all-reduces per forward.

        ``use_rccl`` (default: the group's backend is ``nccl``, i.e. RCCL): the library gets its own
        RCCL communicator over the group's ranks (include/nbx.h nbx_comm_init; collective call) and
        enqueues the all-reduces itself -- no host round trip per BatchNorm.  Otherwise (gloo) the
        library calls back into ``torch.distributed.all_reduce`` on the group.

        ``global_batch``: the number of systems summed over the group's ranks.  When given, a forward
        or rollout makes no collective and no host synchronisation of its own (with RCCL the call can
        then be captured into a HIP graph); it must stay the union of the ranks' batches for every
        call until SyncBN is re-enabled.  When None, every call all-reduces the local batch size
        first (one small collective plus a ``.item()``)."""
        import torch.distributed as dist
        self.disable_sync_batchnorm()
        self._bn_group = group if group is not None else dist.group.WORLD
        self._bn_global_batch = None if global_batch is None else int(global_batch)
        if use_rccl is None:
            use_rccl = dist.get_backend(self._bn_group) == "nccl"
        if use_rccl:
            import ctypes
            ranks = dist.get_process_group_ranks(self._bn_group)
            me = dist.get_rank(self._bn_group)
            uid = [None]
            if me == 0:
                buf = ctypes.create_string_buffer(_lib.COMM_ID_BYTES)
                _lib.check(_lib.lib().nbx_comm_unique_id(buf), "nbx_comm_unique_id")
                uid[0] = buf.raw
            dist.broadcast_object_list(uid, src=ranks[0], group=self._bn_group)
            comm = _lib.c_p()
            dev = torch.cuda.current_device()
            _lib.check(_lib.lib().nbx_comm_init(ctypes.create_string_buffer(uid[0], _lib.COMM_ID_BYTES), len(ranks),
                                                me, dev, ctypes.byref(comm)), "nbx_comm_init")
            self._bn_comm = comm
            # a model dropped without disable_sync_batchnorm() still releases its communicator
            self._bn_comm_fin = weakref.finalize(self, _destroy_comm, comm)
        return self

    def disable_sync_batchnorm(self):
        if self._bn_comm is not None:
            self._bn_comm_fin()      # synchronise, nbx_comm_destroy (runs once)
            self._bn_comm, self._bn_comm_fin = None, None
        self._bn_group = None
        self._bn_global_batch = None
        return self

    def _allreduce_cb(self, buf, count, stream, ctx):
        try:
            import torch.distributed as dist
            ws = self._ws
            off = int(buf) - ws.data_ptr()
            if off < 0 or off + 8 * count > ws.numel() or off % 8:
                raise _lib.NbxError("bn_allreduce: buffer outside the workspace")
            dist.all_reduce(ws[off:off + 8 * count].view(torch.float64), group=self._bn_group)
            return 0
        except Exception:  # reported to the library as a failed hook -> NbxError in the caller
            import traceback
            traceback.print_exc()
            return 1

    def _arm_sync(self, W, B, device):
        """Point the weight struct's hook at the SyncBN callback (or clear it) for one call."""
        if self._bn_group is None or not self._bn_batch():
            W.bn_allreduce = _lib.ALLREDUCE_FN()
            W.bn_comm = None
            W.bn_global_batch = 0
            return
        import torch.distributed as dist
        if self._bn_comm is not None:
            W.bn_comm = self._bn_comm
            W.bn_allreduce = _lib.ALLREDUCE_FN()
        else:
            if self._bn_hook is None:
                self._bn_hook = _lib.ALLREDUCE_FN(self._allreduce_cb)
            W.bn_comm = None
            W.bn_allreduce = self._bn_hook
        if self._bn_global_batch is not None:
            if B > self._bn_global_batch:
                raise ValueError(f"SyncBN: local batch {B} exceeds global_batch {self._bn_global_batch}")
            W.bn_global_batch = self._bn_global_batch
            return
        on_dev = dist.get_backend(self._bn_group) == "nccl"
        nb = torch.tensor([B], dtype=torch.int64, device=device if on_dev else "cpu")
        dist.all_reduce(nb, group=self._bn_group)
        W.bn_global_batch = int(nb.item())

    def _bn_sync_in(self):
        for buf, sh in self._packed[3]:
            sh.copy_(buf)

    def _bn_sync_out(self):
        if self._bn_batch():
            for buf, sh in self._packed[3]:
                buf.copy_(sh)

    def _workspace(self, B, N, device):
        nbytes = _lib.c_sz()
        _lib.check(_lib.lib().nbx_segnn_workspace_bytes(B, N, self.mul, nbytes), "segnn workspace")
        if self._ws is None or self._ws.numel() < nbytes.value or self._ws.device != device:
            self._ws = torch.empty(nbytes.value, dtype=torch.uint8, device=device)
        return self._ws

    def _check_params(self, device):
        for p in self.parameters():
            if not p.is_cuda:
                raise _lib.NbxError("SEGNN HIP path: move the model to the HIP device first")

    # ------------------------------------------------------------ forward
    @staticmethod
    def infer_system_size(num_nodes: int, num_edges: int):
        if num_nodes == 0:
            raise ValueError("empty graph")
        n = num_edges // num_nodes + 1
        if num_edges != num_nodes * (n - 1) or num_nodes % n:
            raise NotImplementedError("native SEGNN needs fully-connected systems of equal size")
        return num_nodes // n, n

    def forward(self, graph):
        """graph: pos [V,3], vel [V,3], mass [V,1], edge_index (build_graph_with_knn: the
        fully-connected pattern, its kNN graphs, or any simple graph inside equal-size systems),
        batch.  Returns [V, 6] in the graph's dtype; computes in fp32."""
        pos = graph.pos
        device = pos.device
        V = pos.shape[0]
        edge_index = graph.edge_index
        from .graph import system_layout
        B, N, fc = system_layout(graph, V, edge_index.shape[1], device)
        out_dtype = pos.dtype
        if out_dtype != torch.float32 and not self._warned_dtype:
            warnings.warn("SEGNN HIP path computes in fp32; inputs are cast", stacklevel=2)
            self._warned_dtype = True
        self._check_params(device)
        f = lambda t: t.detach().to(device=device, dtype=torch.float32).contiguous()
        p, v, m = f(pos), f(graph.vel), f(graph.mass.reshape(-1))
        if use_training_path(self):   # train_dispatch.py: autograd on + trainable params
            # training step (trainer.py:233-358): the forward runs on the native training operators
            # with autograd (segnn_train.py), so loss.backward() reaches every parameter
            # with enable_sync_batchnorm() the step's batch statistics span every rank of the group
            # (segnn_train._SyncBNFn: one all-reduce of the fp64 sums per BatchNorm, forward and backward)
            from . import segnn_train
            return segnn_train.train_forward(self, p, v, m, edge_index).to(out_dtype)
        out = torch.empty(V, 6, device=device, dtype=torch.float32)
        W = self._weights(device)
        ws = self._workspace(B, N, device)
        self._arm_sync(W, B, device)
        self._bn_sync_in()
        if fc:
            _lib.check(_lib.lib().nbx_segnn_forward(
                W, _lib.dev_ptr(p), _lib.dev_ptr(v), _lib.dev_ptr(m), B, N, _lib.dev_ptr(out),
                _lib.dev_ptr(ws), ws.numel(), _lib.stream_ptr(device)), "nbx_segnn_forward")
        else:
            ei = edge_index.to(device=device, dtype=torch.int64).contiguous()
            _lib.check(_lib.lib().nbx_segnn_forward_graph(
                W, _lib.dev_ptr(p), _lib.dev_ptr(v), _lib.dev_ptr(m), B, N, _lib.dev_ptr(ei), ei.shape[1],
                _lib.dev_ptr(out), _lib.dev_ptr(ws), ws.numel(), _lib.stream_ptr(device)),
                "nbx_segnn_forward_graph")
        self._bn_sync_out()
        self._range_check(B, N, device)
        return out.to(out_dtype)

    @torch.no_grad()
    def rollout(self, loc, vel, mass, num_frames: int, absolute: bool = False, num_neighbors=None):
        """Device-resident self-feed (infer_self_feed.py:99-194): loc/vel [B,N,3], mass [B,N,1]
        -> (traj_loc, traj_vel) [B, num_frames, N, 3] fp32.  ``absolute``: the model predicts
        positions (dataset targets other than "pos_dt+vel", infer_self_feed.py:185-186).
        ``num_neighbors``: each frame's graph is build_graph_with_knn's kNN graph of that frame's
        positions (None / N-1: fully connected)."""
        device = loc.device
        self._check_params(device)
        B, N, _ = loc.shape
        f = lambda t: t.detach().to(device=device, dtype=torch.float32).contiguous().clone()
        p, v, m = f(loc), f(vel), f(mass.reshape(B * N))
        tp = torch.empty(B, num_frames, N, 3, device=device, dtype=torch.float32)
        tv = torch.empty_like(tp)
        W = self._weights(device)
        ws = self._workspace(B, N, device)
        self._arm_sync(W, B, device)
        self._bn_sync_in()
        flags = _lib.ROLLOUT_ABSOLUTE if absolute else 0
        if num_neighbors is None or int(num_neighbors) == N - 1:
            _lib.check(_lib.lib().nbx_segnn_rollout(
                W, _lib.dev_ptr(p), _lib.dev_ptr(v), _lib.dev_ptr(m), B, N, num_frames, flags,
                _lib.dev_ptr(tp), _lib.dev_ptr(tv), _lib.dev_ptr(ws), ws.numel(), _lib.stream_ptr(device)),
                "nbx_segnn_rollout")
        else:
            _lib.check(_lib.lib().nbx_segnn_rollout_knn(
                W, _lib.dev_ptr(p), _lib.dev_ptr(v), _lib.dev_ptr(m), B, N, num_frames, flags,
                int(num_neighbors), _lib.dev_ptr(tp), _lib.dev_ptr(tv), _lib.dev_ptr(ws), ws.numel(),
                _lib.stream_ptr(device)), "nbx_segnn_rollout_knn")
        self._bn_sync_out()
        self._range_check(B, N, device)
        return tp, tv

    def _range_check(self, B, N, device):
        """fp16x2 range guard (include/nbx.h nbx_segnn_range_check): NbxError when a tensor-product operand
        of the call left the fp16 range of the split path (or an input was not finite) instead of returning
        non-finite values.  One stream synchronisation per call; skipped while a HIP graph is being
        captured (call ``check_range`` after a replay) and when ``range_check`` is False."""
        if self.range_check and not torch.cuda.is_current_stream_capturing():
            self.check_range(B, N, device)

    def check_range(self, B, N, device=None):
        device = device if device is not None else self._ws.device
        _lib.check(_lib.lib().nbx_segnn_range_check(_lib.dev_ptr(self._ws), self._ws.numel(), B, N, self.mul,
                                                    _lib.stream_ptr(device)), "segnn")
