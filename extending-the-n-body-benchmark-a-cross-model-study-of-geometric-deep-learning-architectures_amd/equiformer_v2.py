"""EquiformerV2_nbody — drop-in for models/equiformer_v2/architecture/equiformer_v2_nbody.py with a
HIP forward (csrc/eqv2.hip).

The module tree, parameter / buffer names and shapes, and the order in which parameters draw from
the RNG (construction, then ``_init_weights`` and the radial-function re-initialisation,
equiformer_v2_nbody.py:388-389,585-606) follow the reference, so reference checkpoints load with
``load_state_dict`` and ``torch.manual_seed(s)`` gives the reference's weights.  ``forward(data,
batch)`` accepts the tuple input of helper_scripts/infer_self_feed.py:178-181 ``(pos, vel, force,
charges, pos)`` or an object with ``pos`` / ``vel`` (/ ``x``) and returns ``[B*N, 6]`` (delta pos |
vel); ``rollout`` runs the self-feed loop device-resident.  Eval-mode semantics (no alpha dropout,
no drop path: the self-feed path runs ``model.eval()``, nbody_utils.py:1372).

init_edge_rot_mat draws one random vector per edge from torch's RNG (edge_rot_mat.py:21); the
native path draws them on the device from a counter-based hash of (``gauge_seed``, call counter,
edge), or takes them explicitly (``forward(..., gauge=...)``).
"""
from __future__ import annotations

import copy
import math
from typing import List

import torch
from torch import nn

from . import _lib
from .train_dispatch import use_training_path
from . import so3

__all__ = ["EquiformerV2_nbody"]

AVG_DEGREE = 23.395238876342773   # equiformer_v2_nbody.py:36
PROJECTION_DIM = 1024             # equiformer_v2_nbody.py:219


# ----------------------------------------------------------------------------- parameter containers
class _CoefficientMapping(nn.Module):
    """CoefficientMappingModule (so3.py:30-115): buffers only."""

    def __init__(self, lmax_list, mmax_list):
        super().__init__()
        self.lmax_list, self.mmax_list = list(lmax_list), list(mmax_list)
        for k, v in so3.coefficient_mapping(lmax_list, mmax_list).items():
            self.register_buffer(k, v)


class _SO3Rotation(nn.Module):
    def __init__(self, lmax):
        super().__init__()
        self.lmax = lmax
        self.mapping = _CoefficientMapping([lmax], [lmax])


class _SO3Grid(nn.Module):
    def __init__(self, lmax, mmax):
        super().__init__()
        self.lmax, self.mmax = lmax, mmax
        self.mapping = _CoefficientMapping([lmax], [lmax])
        to, fr = so3.so3_grid(lmax, mmax)
        self.register_buffer("to_grid_mat", to)
        self.register_buffer("from_grid_mat", fr)


class _ModuleListInfo(nn.ModuleList):
    def __init__(self, info_str, modules=None):
        super().__init__(modules)
        self.info_str = str(info_str)


class _RadialFunction(nn.Module):
    """RadialFunction (radial_function.py:5-32)."""

    def __init__(self, channels_list):
        super().__init__()
        mods, cin = [], channels_list[0]
        for i in range(1, len(channels_list)):
            mods.append(nn.Linear(cin, int(channels_list[i]), bias=True))
            cin = int(channels_list[i])
            if i == len(channels_list) - 1:
                break
            mods.append(nn.LayerNorm(channels_list[i]))
            mods.append(nn.SiLU())
        self.net = nn.Sequential(*mods)


class _SO2mConvolution(nn.Module):
    def __init__(self, m, sphere_channels, m_output_channels, lmax_list, mmax_list):
        super().__init__()
        nch = sum((l - m + 1 if mm >= m else 0) * sphere_channels for l, mm in zip(lmax_list, mmax_list))
        self.fc = nn.Linear(nch, 2 * m_output_channels * (nch // sphere_channels), bias=False)
        self.fc.weight.data.mul_(1 / math.sqrt(2))


class _SO2Convolution(nn.Module):
    """SO2_Convolution (so2_ops.py:78-156)."""

    def __init__(self, sphere_channels, m_output_channels, lmax_list, mmax_list, mappingReduced,
                 internal_weights=True, edge_channels_list=None, extra_m0_output_channels=None):
        super().__init__()
        self.mappingReduced = mappingReduced
        self.extra_m0_output_channels = extra_m0_output_channels
        nm0 = sum((l + 1) * sphere_channels for l in lmax_list)
        out0 = m_output_channels * (nm0 // sphere_channels) + (extra_m0_output_channels or 0)
        self.fc_m0 = nn.Linear(nm0, out0)
        nrad = self.fc_m0.in_features
        self.so2_m_conv = nn.ModuleList()
        for m in range(1, max(mmax_list) + 1):
            self.so2_m_conv.append(_SO2mConvolution(m, sphere_channels, m_output_channels, lmax_list, mmax_list))
            nrad += self.so2_m_conv[-1].fc.in_features
        self.rad_func = None
        if not internal_weights:
            self.rad_func = _RadialFunction(copy.deepcopy(edge_channels_list) + [int(nrad)])


class _SO3LinearV2(nn.Module):
    """SO3_LinearV2 (so3.py:695-745)."""

    def __init__(self, in_features, out_features, lmax):
        super().__init__()
        self.in_features, self.out_features, self.lmax = in_features, out_features, lmax
        self.weight = nn.Parameter(torch.randn(lmax + 1, out_features, in_features))
        bound = 1 / math.sqrt(in_features)
        nn.init.uniform_(self.weight, -bound, bound)
        self.bias = nn.Parameter(torch.zeros(out_features))
        self.register_buffer("expand_index", torch.tensor([float(l) for l in range(lmax + 1)
                                                           for _ in range(2 * l + 1)]))


class _RMSNormSH(nn.Module):
    """EquivariantRMSNormArraySphericalHarmonicsV2 (layer_norm.py:327-441), affine, centering."""

    def __init__(self, lmax, num_channels, eps=1e-5):
        super().__init__()
        self.lmax, self.num_channels, self.eps = lmax, num_channels, eps
        self.affine_weight = nn.Parameter(torch.ones(lmax + 1, num_channels))
        self.affine_bias = nn.Parameter(torch.zeros(num_channels))
        self.register_buffer("expand_index", torch.tensor([float(l) for l in range(lmax + 1)
                                                           for _ in range(2 * l + 1)]))
        bal = torch.tensor([[1.0 / (2 * l + 1) / (lmax + 1)] for l in range(lmax + 1) for _ in range(2 * l + 1)])
        self.register_buffer("balance_degree_weight", bal)


class _GraphAttention(nn.Module):
    """SO2EquivariantGraphAttention (transformer_block.py:22-224), separable S2 activation."""

    def __init__(self, sphere_channels, hidden_channels, num_heads, attn_alpha_channels, attn_value_channels,
                 output_channels, lmax_list, mmax_list, SO3_rotation, mappingReduced, SO3_grid, max_num_elements,
                 edge_channels_list, use_atom_edge_embedding=True, alpha_drop=0.0):
        super().__init__()
        self.num_heads, self.attn_alpha_channels = num_heads, attn_alpha_channels
        self.attn_value_channels, self.output_channels = attn_value_channels, output_channels
        self.SO3_rotation, self.mappingReduced, self.SO3_grid = SO3_rotation, mappingReduced, SO3_grid
        ecl = copy.deepcopy(edge_channels_list)
        if use_atom_edge_embedding:
            self.source_embedding = nn.Embedding(max_num_elements, ecl[-1])
            self.target_embedding = nn.Embedding(max_num_elements, ecl[-1])
            nn.init.uniform_(self.source_embedding.weight.data, -0.001, 0.001)
            nn.init.uniform_(self.target_embedding.weight.data, -0.001, 0.001)
            ecl[0] = ecl[0] + 2 * ecl[-1]
        else:
            self.source_embedding = self.target_embedding = None
        extra = num_heads * attn_alpha_channels + hidden_channels
        self.so2_conv_1 = _SO2Convolution(2 * sphere_channels, hidden_channels, lmax_list, mmax_list, mappingReduced,
                                          internal_weights=False, edge_channels_list=ecl,
                                          extra_m0_output_channels=extra)
        self.alpha_norm = nn.LayerNorm(attn_alpha_channels)
        self.alpha_dot = nn.Parameter(torch.randn(num_heads, attn_alpha_channels))
        std = 1.0 / math.sqrt(attn_alpha_channels)
        nn.init.uniform_(self.alpha_dot, -std, std)
        self.alpha_drop = alpha_drop
        self.so2_conv_2 = _SO2Convolution(hidden_channels, num_heads * attn_value_channels, lmax_list, mmax_list,
                                          mappingReduced, internal_weights=True)
        self.proj = _SO3LinearV2(num_heads * attn_value_channels, output_channels, lmax=lmax_list[0])


class _FeedForward(nn.Module):
    """FeedForwardNetwork (transformer_block.py:373-471), separable S2 activation."""

    def __init__(self, sphere_channels, hidden_channels, output_channels, lmax_list, SO3_grid):
        super().__init__()
        self.SO3_grid = SO3_grid
        lmax = max(lmax_list)
        self.so3_linear_1 = _SO3LinearV2(sphere_channels * len(lmax_list), hidden_channels, lmax=lmax)
        self.gating_linear = nn.Linear(sphere_channels * len(lmax_list), hidden_channels)
        self.so3_linear_2 = _SO3LinearV2(hidden_channels, output_channels, lmax=lmax)


class _TransBlock(nn.Module):
    """TransBlockV2 (transformer_block.py:533-667)."""

    def __init__(self, C, H, nh, na, nv, F, lmax_list, mmax_list, SO3_rotation, mappingReduced, SO3_grid,
                 max_num_elements, edge_channels_list, use_atom_edge_embedding, alpha_drop, drop_path_rate):
        super().__init__()
        lmax = max(lmax_list)
        self.norm_1 = _RMSNormSH(lmax, C)
        self.ga = _GraphAttention(C, H, nh, na, nv, C, lmax_list, mmax_list, SO3_rotation, mappingReduced, SO3_grid,
                                  max_num_elements, edge_channels_list, use_atom_edge_embedding, alpha_drop)
        self.drop_path_rate = drop_path_rate
        self.norm_2 = _RMSNormSH(lmax, C)
        self.ffn = _FeedForward(C, F, C, lmax_list, SO3_grid)


class _EdgeDegreeEmbedding(nn.Module):
    """EdgeDegreeEmbedding (input_block.py:11-81)."""

    def __init__(self, C, lmax_list, mmax_list, SO3_rotation, mappingReduced, max_num_elements, edge_channels_list,
                 use_atom_edge_embedding):
        super().__init__()
        self.SO3_rotation, self.mappingReduced = SO3_rotation, mappingReduced
        ecl = copy.deepcopy(edge_channels_list)
        if use_atom_edge_embedding:
            self.source_embedding = nn.Embedding(max_num_elements, ecl[-1])
            self.target_embedding = nn.Embedding(max_num_elements, ecl[-1])
            nn.init.uniform_(self.source_embedding.weight.data, -0.001, 0.001)
            nn.init.uniform_(self.target_embedding.weight.data, -0.001, 0.001)
            ecl[0] = ecl[0] + 2 * ecl[-1]
        m0 = int(mappingReduced.m_size[0].item())
        self.rad_func = _RadialFunction(ecl + [m0 * C])
        self.rescale_factor = AVG_DEGREE


# ----------------------------------------------------------------------------- the model
class EquiformerV2_nbody(nn.Module):
    """EquiformerV2_nbody (equiformer_v2_nbody.py:57-389): constructor arguments and defaults of the
    reference; the fused forward covers its C4 / inference configurations (include/nbx.h,
    EquiformerV2 section), the composed one (eqv2_train.py) every single-resolution lmax <= 6
    including the constructor default lmax 6 / mmax 2."""

    def __init__(self, device=None, use_pbc=False, regress_forces=True, otf_graph=True, max_neighbors=5,
                 max_radius=4096, max_num_elements=90, num_layers=12, attn_hidden_channels=128, sphere_channels=128,
                 num_heads=8, attn_alpha_channels=32, attn_value_channels=16, ffn_hidden_channels=512,
                 norm_type="rms_norm_sh", lmax_list: List[int] = [6], mmax_list: List[int] = [2],
                 grid_resolution=None, num_sphere_samples=128, edge_channels=128, use_atom_edge_embedding=True,
                 share_atom_edge_embedding=False, use_m_share_rad=False, distance_function="projection",
                 num_distance_basis=512, attn_activation="scaled_silu", use_s2_act_attn=False, use_attn_renorm=True,
                 ffn_activation="scaled_silu", use_gate_act=False, use_grid_mlp=False, use_sep_s2_act=True,
                 alpha_drop=0.1, drop_path_rate=0.05, proj_drop=0.0, weight_init="normal"):
        super().__init__()
        self.use_pbc, self.regress_forces, self.otf_graph = use_pbc, regress_forces, otf_graph
        self.max_neighbors, self.max_radius, self.cutoff = max_neighbors, max_radius, max_radius
        self.max_num_elements, self.num_layers = max_num_elements, num_layers
        self.sphere_channels, self.attn_hidden_channels = sphere_channels, attn_hidden_channels
        self.num_heads, self.attn_alpha_channels = num_heads, attn_alpha_channels
        self.attn_value_channels, self.ffn_hidden_channels = attn_value_channels, ffn_hidden_channels
        self.norm_type, self.lmax_list, self.mmax_list = norm_type, list(lmax_list), list(mmax_list)
        self.grid_resolution, self.num_sphere_samples = grid_resolution, num_sphere_samples
        self.edge_channels, self.use_atom_edge_embedding = edge_channels, use_atom_edge_embedding
        self.share_atom_edge_embedding, self.use_m_share_rad = share_atom_edge_embedding, use_m_share_rad
        self.distance_function, self.num_distance_basis = distance_function, num_distance_basis
        self.attn_activation, self.use_s2_act_attn, self.use_attn_renorm = attn_activation, use_s2_act_attn, use_attn_renorm
        self.ffn_activation, self.use_gate_act, self.use_grid_mlp = ffn_activation, use_gate_act, use_grid_mlp
        self.use_sep_s2_act = use_sep_s2_act
        self.alpha_drop, self.drop_path_rate, self.proj_drop = alpha_drop, drop_path_rate, proj_drop
        self.weight_init = weight_init
        assert weight_init in ("normal", "uniform")
        reasons = []
        if list(lmax_list) != [2] or list(mmax_list) != [1]:
            reasons.append("lmax_list [2], mmax_list [1]")
        if norm_type != "rms_norm_sh" or distance_function != "projection" or grid_resolution is not None:
            reasons.append('norm_type "rms_norm_sh", distance_function "projection", default grid resolution')
        if (not use_atom_edge_embedding or share_atom_edge_embedding or use_m_share_rad or use_s2_act_attn
                or use_gate_act or use_grid_mlp or not use_sep_s2_act or not use_attn_renorm):
            reasons.append("per-module atom edge embeddings, separable S2 activations, attention re-norm")
        if (sphere_channels not in (32, 64) or attn_hidden_channels not in (32, 64)
                or ffn_hidden_channels not in (32, 64) or edge_channels not in (32, 64)
                or num_heads * attn_value_channels not in (8, 16, 32) or num_heads > 8 or attn_alpha_channels > 16):
            reasons.append("C, H, F, edge channels in {32, 64}; heads*value in {8, 16, 32}")
        if num_layers > _lib.EQV2_MAX_LAYERS:
            reasons.append(f"num_layers <= {_lib.EQV2_MAX_LAYERS}")
        self._native_reason = ("native EquiformerV2 needs " + "; ".join(reasons)) if reasons else None
        # the composed path (eqv2_train.py on the general-degree operators, csrc/eqv2_general.hip) runs
        # every single-resolution lmax <= 6 with the reference's default module choices
        general = []
        if len(lmax_list) != 1 or len(mmax_list) != 1:
            general.append("one resolution (len(lmax_list) == 1)")
        elif not 0 <= mmax_list[0] <= lmax_list[0] <= so3.LMAX:
            general.append(f"0 <= mmax <= lmax <= {so3.LMAX}")
        if norm_type != "rms_norm_sh" or distance_function != "projection" or grid_resolution is not None:
            general.append('norm_type "rms_norm_sh", distance_function "projection", default grid resolution')
        if (not use_atom_edge_embedding or share_atom_edge_embedding or use_m_share_rad or use_s2_act_attn
                or use_gate_act or use_grid_mlp or not use_sep_s2_act or not use_attn_renorm):
            general.append("per-module atom edge embeddings, separable S2 activations, attention re-norm")
        if edge_channels > 1024 or attn_alpha_channels > 1024:
            general.append("edge / alpha channels <= 1024")
        self._general_reason = ("EquiformerV2 needs " + "; ".join(general)) if general else None
        if self._general_reason:
            raise NotImplementedError(self._general_reason)
        self.layout = so3.Layout(lmax_list[0], mmax_list[0])
        # composed path at lmax 2 / mmax 1: the general-degree operators (default; measured 7 % faster in
        # the training step, profiles/r04/eqv2_train_glue) or the lmax-2 ones (specialised_ops = True,
        # or NBX_EQV2_SPECIALISED=1)
        import os
        self.specialised_ops = os.environ.get("NBX_EQV2_SPECIALISED", "0") == "1"
        self.force_general_ops = False
        self._wtab = None

        C, He = sphere_channels, edge_channels
        self.num_resolutions = len(self.lmax_list)
        self.sphere_channels_all = self.num_resolutions * C
        self.sphere_embedding = nn.Embedding(max_num_elements, self.sphere_channels_all)
        self.velocity_embedding = nn.Linear(3, 3 * C)
        if distance_function != "projection":
            raise NotImplementedError("distance_function 'projection' only")
        self.distance_expansion = nn.Linear(1, PROJECTION_DIM)
        self.edge_channels_list = [PROJECTION_DIM, He, He]
        self.source_embedding, self.target_embedding = None, None
        self.SO3_rotation = nn.ModuleList([_SO3Rotation(l) for l in self.lmax_list])
        self.mappingReduced = _CoefficientMapping(self.lmax_list, self.mmax_list)
        L = max(self.lmax_list)
        self.SO3_grid = _ModuleListInfo(f"({L}, {L})")
        for l in range(L + 1):
            self.SO3_grid.append(nn.ModuleList([_SO3Grid(l, m) for m in range(L + 1)]))
        self.edge_degree_embedding = _EdgeDegreeEmbedding(C, self.lmax_list, self.mmax_list, self.SO3_rotation,
                                                          self.mappingReduced, max_num_elements,
                                                          self.edge_channels_list, use_atom_edge_embedding)
        self.blocks = nn.ModuleList([
            _TransBlock(C, attn_hidden_channels, num_heads, attn_alpha_channels, attn_value_channels,
                        ffn_hidden_channels, self.lmax_list, self.mmax_list, self.SO3_rotation, self.mappingReduced,
                        self.SO3_grid, max_num_elements, self.edge_channels_list, use_atom_edge_embedding,
                        alpha_drop, drop_path_rate) for _ in range(num_layers)])
        self.norm = _RMSNormSH(L, C)
        self.energy_block = _FeedForward(C, ffn_hidden_channels, 1, self.lmax_list, self.SO3_grid)
        if regress_forces:
            self.force_block = _GraphAttention(C, attn_hidden_channels, num_heads, attn_alpha_channels,
                                               attn_value_channels, 2, self.lmax_list, self.mmax_list,
                                               self.SO3_rotation, self.mappingReduced, self.SO3_grid,
                                               max_num_elements, self.edge_channels_list, use_atom_edge_embedding)
        self.vel_block = _GraphAttention(C, attn_hidden_channels, num_heads, attn_alpha_channels, attn_value_channels,
                                         1, self.lmax_list, self.mmax_list, self.SO3_rotation, self.mappingReduced,
                                         self.SO3_grid, max_num_elements, self.edge_channels_list,
                                         use_atom_edge_embedding)
        self.apply(self._init_weights)
        self.apply(self._uniform_init_rad_func_linear_weights)
        self.gauge_seed = 0
        self._calls = 0
        self._packed = None
        self._ws = None

    # ------------------------------------------------------------ initialisation (reference :585-606)
    def _init_weights(self, m):
        if isinstance(m, (nn.Linear, _SO3LinearV2)):
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
            if self.weight_init == "normal":
                nn.init.normal_(m.weight, 0, 1 / math.sqrt(m.in_features))
        elif isinstance(m, nn.LayerNorm):
            nn.init.constant_(m.bias, 0)
            nn.init.constant_(m.weight, 1.0)

    def _uniform_init_rad_func_linear_weights(self, m):
        if isinstance(m, _RadialFunction):
            m.apply(self._uniform_init_linear_weights)

    @staticmethod
    def _uniform_init_linear_weights(m):
        if isinstance(m, nn.Linear):
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
            std = 1 / math.sqrt(m.in_features)
            nn.init.uniform_(m.weight, -std, std)

    @property
    def num_params(self):
        return sum(p.numel() for p in self.parameters())

    def get_model_size(self):
        return self.sphere_channels

    # ------------------------------------------------------------ packing (include/nbx.h, EquiformerV2)
    def _param_version(self):
        return tuple((p.data_ptr(), p._version) for p in self.parameters())

    @staticmethod
    def _image(W):
        from .segnn import SEGNN
        rows = W.shape[0]
        return SEGNN.frag_image_x3([(W.float(), W.shape[1])], None, -(-rows // 32), 32)

    @classmethod
    def _image_chunk_major(cls, W):
        """[N/32][K/32] blocks -> [K/32][N/32] (include/nbx.h: so2_conv_1 images)."""
        img = cls._image(W)
        nt, kc = img.shape[0], W.shape[1] // 32
        return img.reshape(nt, kc, -1).transpose(0, 1).contiguous()

    @staticmethod
    def _image_h2(W, chunk_major=False):
        """fp16x2 image of W (include/nbx.h "fp16x2 images", the _image block order, optionally chunk-major)
        and its descale 1 / s as a 0-d float64 tensor."""
        from .segnn import SEGNN
        W = W.float()
        s = SEGNN.h2_scale(W)
        rows = W.shape[0]
        img = SEGNN.frag_image_h2([(W, W.shape[1])], None, -(-rows // 32), 32, s)
        if chunk_major:
            nt, kc = img.shape[0], W.shape[1] // 32
            img = img.reshape(nt, kc, -1).transpose(0, 1).contiguous()
        return img, torch.tensor(1.0 / s, dtype=torch.float64)

    def packed_tensors(self, device):
        """Every device tensor the C-ABI weight struct points at, keyed by struct path."""
        C, He = self.sphere_channels, self.edge_channels
        f32 = dict(device=device, dtype=torch.float32)
        d64 = lambda t: t.detach().to(device="cpu", dtype=torch.float64)
        v = lambda t: t.detach().to(**f32).contiguous()
        pad = lambda t, n: torch.nn.functional.pad(t, (0, n - t.shape[0])) if t.shape[0] < n else t
        c32 = lambda n: -(-n // 32) * 32
        P = {}
        de_w, de_b = d64(self.distance_expansion.weight)[:, 0], d64(self.distance_expansion.bias)

        def radial(prefix, rad, src_emb, tgt_emb, permute):
            net = rad.net
            W0, b0 = d64(net[0].weight), d64(net[0].bias)
            Wd, Ws, Wt = W0[:, :PROJECTION_DIM], W0[:, PROJECTION_DIM:PROJECTION_DIM + He], W0[:, PROJECTION_DIM + He:]
            P[prefix + "a"] = v(Wd @ de_w)
            P[prefix + "c"] = v(Wd @ de_b + b0)
            P[prefix + "us"] = v(d64(src_emb.weight) @ Ws.T)
            P[prefix + "ut"] = v(d64(tgt_emb.weight) @ Wt.T)
            P[prefix + "ln1_w"], P[prefix + "ln1_b"] = v(net[1].weight), v(net[1].bias)
            P[prefix + "w1"], P[prefix + "b1"] = v(net[3].weight), v(net[3].bias)
            P[prefix + "ln2_w"], P[prefix + "ln2_b"] = v(net[4].weight), v(net[4].bias)
            P[prefix + "w1_h2"], P[prefix + "w1_sinv"] = self._image_h2(net[3].weight.detach().to(device))
            W2, b2 = net[6].weight.detach(), net[6].bias.detach()
            if permute:
                n = torch.arange(10 * C)
                cb, g, i = n // 160, (n % 160) // 32, n % 32
                perm = g * 2 * C + 32 * cb + i
                P[prefix + "w2_x3"] = self._image(W2[perm].to(device)).to(device)
                P[prefix + "b2"] = v(b2[perm])
                return W2[perm]
            P[prefix + "w2"], P[prefix + "b2"] = v(W2), v(b2)
            P[prefix + "w2_h2"], P[prefix + "w2_sinv"] = self._image_h2(W2.to(device))
            return None

        def attn(prefix, A):
            W2p = radial(prefix + "rad.", A.so2_conv_1.rad_func, A.source_embedding, A.target_embedding, True)
            # fp16x2 images of the five split-precision GEMMs (include/nbx.h nbx_eqv2_attn "fp16x2 images")
            P[prefix + "w2_h2"], P[prefix + "w2_sinv"] = self._image_h2(W2p.to(device))
            P[prefix + "fc0_h2"], P[prefix + "fc0_sinv"] = self._image_h2(
                A.so2_conv_1.fc_m0.weight.detach().to(device), chunk_major=True)
            P[prefix + "fc1_h2"], P[prefix + "fc1_sinv"] = self._image_h2(
                A.so2_conv_1.so2_m_conv[0].fc.weight.detach().to(device), chunk_major=True)
            P[prefix + "c20_h2"], P[prefix + "c20_sinv"] = self._image_h2(A.so2_conv_2.fc_m0.weight.detach().to(device))
            P[prefix + "c21_h2"], P[prefix + "c21_sinv"] = self._image_h2(
                A.so2_conv_2.so2_m_conv[0].fc.weight.detach().to(device))
            fc0 = A.so2_conv_1.fc_m0
            n0 = c32(fc0.out_features)
            P[prefix + "fc0_x3"] = self._image_chunk_major(fc0.weight.detach().to(device))
            P[prefix + "fc0_b"] = v(pad(fc0.bias.detach(), n0))
            P[prefix + "fc1_x3"] = self._image_chunk_major(A.so2_conv_1.so2_m_conv[0].fc.weight.detach().to(device))
            c20 = A.so2_conv_2.fc_m0
            P[prefix + "c20_x3"] = self._image(c20.weight.detach().to(device))
            P[prefix + "c20_b"] = v(pad(c20.bias.detach(), c32(c20.out_features)))
            P[prefix + "c21_x3"] = self._image(A.so2_conv_2.so2_m_conv[0].fc.weight.detach().to(device))
            P[prefix + "alpha_norm_w"], P[prefix + "alpha_norm_b"] = v(A.alpha_norm.weight), v(A.alpha_norm.bias)
            P[prefix + "alpha_dot"] = v(A.alpha_dot)
            P[prefix + "proj_t"] = v(A.proj.weight.transpose(1, 2))       # [3][nh nv][Cout]
            P[prefix + "proj_b"] = v(A.proj.bias)

        radial("edge_degree.", self.edge_degree_embedding.rad_func, self.edge_degree_embedding.source_embedding,
               self.edge_degree_embedding.target_embedding, False)
        attn("force.", self.force_block)
        for i, blk in enumerate(self.blocks):
            p = f"blocks.{i}."
            attn(p + "ga.", blk.ga)
            P[p + "norm1_w"], P[p + "norm1_b"] = v(blk.norm_1.affine_weight), v(blk.norm_1.affine_bias)
            P[p + "norm2_w"], P[p + "norm2_b"] = v(blk.norm_2.affine_weight), v(blk.norm_2.affine_bias)
            P[p + "gate_t"], P[p + "gate_b"] = v(blk.ffn.gating_linear.weight.T), v(blk.ffn.gating_linear.bias)
            P[p + "lin1_t"], P[p + "lin1_b"] = v(blk.ffn.so3_linear_1.weight.transpose(1, 2)), v(blk.ffn.so3_linear_1.bias)
            P[p + "lin2_t"], P[p + "lin2_b"] = v(blk.ffn.so3_linear_2.weight.transpose(1, 2)), v(blk.ffn.so3_linear_2.bias)
        P["norm_w"], P["norm_b"] = v(self.norm.affine_weight), v(self.norm.affine_bias)
        P["sphere_emb"] = v(self.sphere_embedding.weight)
        P["vel_t"], P["vel_b"] = v(self.velocity_embedding.weight.T), v(self.velocity_embedding.bias)
        ga, gf = self.SO3_grid[2][1], self.SO3_grid[2][2]
        P["grid_attn_to"] = v(ga.to_grid_mat.reshape(-1, ga.to_grid_mat.shape[-1]))
        P["grid_attn_from"] = v(ga.from_grid_mat.reshape(-1, ga.from_grid_mat.shape[-1]))
        P["grid_ffn_to"] = v(gf.to_grid_mat.reshape(-1, gf.to_grid_mat.shape[-1]))
        P["grid_ffn_from"] = v(gf.from_grid_mat.reshape(-1, gf.from_grid_mat.shape[-1]))
        return {k: t.to(device).contiguous() for k, t in P.items()}

    def pack_weights(self, device):
        P = self.packed_tensors(device)
        W = _lib.Eqv2Weights()
        W.sphere_channels, W.attn_hidden, W.num_heads = self.sphere_channels, self.attn_hidden_channels, self.num_heads
        W.alpha_channels, W.value_channels = self.attn_alpha_channels, self.attn_value_channels
        W.ffn_hidden, W.edge_channels, W.num_layers = self.ffn_hidden_channels, self.edge_channels, self.num_layers
        W.num_elements = self.max_num_elements

        def fill(struct, prefix):
            for name, typ in struct._fields_:
                if isinstance(getattr(struct, name), ctypes_struct_types()):
                    fill(getattr(struct, name), prefix + name + ".")
                elif typ is _lib.c_f:   # the fp16x2 images' descale factors
                    setattr(struct, name, float(P.get(prefix + name, 1.0)))
                elif prefix + name in P:
                    setattr(struct, name, P[prefix + name].data_ptr())

        fill(W, "")
        for i in range(self.num_layers):
            fill(W.blocks[i], f"blocks.{i}.")
        self._packed = (self._param_version(), W, P)
        return W

    def _weights(self, device):
        if self._native_reason:
            raise NotImplementedError(self._native_reason)
        if self._packed is None or self._packed[0] != self._param_version() or \
                next(iter(self._packed[2].values())).device != device:
            self.pack_weights(device)
        return self._packed[1]

    def _workspace(self, W, B, N, device):
        n = _lib.c_sz()
        _lib.check(_lib.lib().nbx_eqv2_workspace_bytes(W, B, N, n), "eqv2 workspace")
        if self._ws is None or self._ws.numel() < n.value or self._ws.device != device:
            self._ws = None
            self._ws = torch.empty(n.value, dtype=torch.uint8, device=device)
        return self._ws

    def uses_general_ops(self):
        """True when the composed path runs on the general-degree operators (nbx_eqv2_wigner /
        rotate_general / rms_norm_general, m-primary edge irreps) instead of the lmax 2 / mmax 1 ones:
        always outside lmax 2 / mmax 1 and C <= 128, and there unless ``specialised_ops`` is set."""
        lmax2 = (self.layout.lmax, self.layout.mmax) == (2, 1) and self.sphere_channels <= 128
        return not lmax2 or bool(self.force_general_ops) or not self.specialised_ops

    def wigner_table(self, device):
        """so3.wigner_table(lmax) on ``device`` (the probe constants of nbx_eqv2_wigner), cached."""
        if self._wtab is None or self._wtab.device != device:
            n = _lib.c_i64()
            _lib.check(_lib.lib().nbx_eqv2_wigner_table_floats(self.layout.lmax, n), "nbx_eqv2_wigner_table_floats")
            t = so3.wigner_table(self.layout.lmax)
            if n.value and t.numel() != n.value:
                raise RuntimeError("EquiformerV2: Wigner table size disagrees with the library")
            self._wtab = t.to(device)
        return self._wtab

    def _composed(self, p, vv, q, B, N, g, seed, frame=0):
        from . import eqv2_train
        return eqv2_train.train_forward(self, p, vv, q, B, N, g, seed, frame)

    # ------------------------------------------------------------ forward
    def forward(self, data, batch=None, gauge=None):
        """equiformer_v2_nbody.py:392-575 -> [B*N, 6] (delta pos | vel)."""
        if hasattr(data, "pos"):
            pos = data.pos
            vel = data.vel if hasattr(data, "vel") else torch.zeros_like(pos)
            x = getattr(data, "x", None)
            if x is not None and x.shape[1] > 0:
                charges = torch.clamp(x[:, 0], 0, self.max_num_elements - 1)
            else:
                charges = torch.ones(pos.shape[0], device=pos.device)
            if batch is None:
                batch = getattr(data, "batch", None)
        else:
            pos, vel, _, charges, _ = data
        V = pos.shape[0]
        B = int(batch.max().item()) + 1 if batch is not None else 1
        N = V // B
        device = pos.device
        f = lambda t: t.detach().to(device=device, dtype=torch.float32).contiguous()
        p, vv, q = f(pos), f(vel), f(charges.reshape(-1))
        g = None
        if gauge is not None:
            g = f(gauge)
            if g.shape != (V * (N - 1), 3):
                raise ValueError("gauge must be [B*N*(N-1), 3]")
        seed = (int(self.gauge_seed) * 0x100000001B3 + self._calls) & 0xFFFFFFFFFFFFFFFF
        if use_training_path(self):   # train_dispatch.py: autograd on + trainable params
            # training step: native operators under autograd (eqv2_train.py)
            self._calls += 1
            return self._composed(p, vv, q, B, N, g, seed).to(pos.dtype)
        if self._native_reason:
            # no fused kernels for this configuration (e.g. the reference default lmax 6 / mmax 2):
            # the same native operators, composed, without autograd
            self._calls += 1
            with torch.no_grad():
                return self._composed(p, vv, q, B, N, g, seed).to(pos.dtype)
        out = torch.empty(V, 6, device=device, dtype=torch.float32)
        W = self._weights(device)
        ws = self._workspace(W, B, N, device)
        self._calls += 1
        _lib.check(_lib.lib().nbx_eqv2_forward(W, _lib.dev_ptr(p), _lib.dev_ptr(vv), _lib.dev_ptr(q), B, N,
                                               _lib.dev_ptr(g) if g is not None else None, seed, _lib.dev_ptr(out),
                                               _lib.dev_ptr(ws), ws.numel(), _lib.stream_ptr(device)),
                   "nbx_eqv2_forward")
        self._range_check(W, ws, B, N, device)
        return out.to(pos.dtype)

    def _range_check(self, W, ws, B, N, device):
        """fp16x2 range guard (include/nbx.h nbx_eqv2_range_check): NbxError instead of non-finite results when a
        GEMM operand leaves the fp16 range of the split path; one stream synchronisation per call, skipped while a
        HIP graph is captured and when ``range_check`` is False."""
        if getattr(self, "range_check", True) and not torch.cuda.is_current_stream_capturing():
            _lib.check(_lib.lib().nbx_eqv2_range_check(W, _lib.dev_ptr(ws), ws.numel(), B, N, _lib.stream_ptr(device)),
                       "eqv2")

    @torch.no_grad()
    def rollout(self, loc, vel, mass, num_frames: int, absolute: bool = False, seed=None):
        """Device-resident self-feed through the tuple branch (infer_self_feed.py:99-194)."""
        device = loc.device
        B, N, _ = loc.shape
        f = lambda t: t.detach().to(device=device, dtype=torch.float32).contiguous().clone()
        p, v, m = f(loc), f(vel), f(mass.reshape(B * N))
        tp = torch.empty(B, num_frames, N, 3, device=device, dtype=torch.float32)
        tv = torch.empty_like(tp)
        if self._native_reason:
            # composed path: frame f draws its gauges from (seed, f - 1) as nbx_eqv2_rollout does
            if seed is None:
                seed = (int(self.gauge_seed) * 0x100000001B3 + self._calls) & 0xFFFFFFFFFFFFFFFF
                self._calls += 1
            tp[:, 0], tv[:, 0] = p, v
            p, v = p.reshape(B * N, 3), v.reshape(B * N, 3)
            for f in range(1, num_frames):
                pred = self._composed(p, v, m, B, N, None, int(seed), f - 1)
                p = pred[:, :3].contiguous() if absolute else p + pred[:, :3]
                v = pred[:, 3:].contiguous()
                tp[:, f], tv[:, f] = p.view(B, N, 3), v.view(B, N, 3)
            return tp, tv
        W = self._weights(device)
        ws = self._workspace(W, B, N, device)
        if seed is None:
            seed = (int(self.gauge_seed) * 0x100000001B3 + self._calls) & 0xFFFFFFFFFFFFFFFF
            self._calls += 1
        _lib.check(_lib.lib().nbx_eqv2_rollout(W, _lib.dev_ptr(p), _lib.dev_ptr(v), _lib.dev_ptr(m), B, N, num_frames,
                                               _lib.ROLLOUT_ABSOLUTE if absolute else 0, int(seed), _lib.dev_ptr(tp),
                                               _lib.dev_ptr(tv), _lib.dev_ptr(ws), ws.numel(),
                                               _lib.stream_ptr(device)), "nbx_eqv2_rollout")
        self._range_check(W, ws, B, N, device)
        return tp, tv


def ctypes_struct_types():
    import ctypes
    return (ctypes.Structure,)
