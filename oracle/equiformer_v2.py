"""torch float64 restatement of the EquiformerV2 N-body forward — TEST ORACLE ONLY.

Follows (all under models/equiformer_v2/architecture/):
* EquiformerV2_nbody._forward_internal          equiformer_v2_nbody.py:428-575 (tuple input branch
                                                 forward:392-426; atomic numbers = mass.int())
* init_edge_rot_mat (random gauge supplied)     edge_rot_mat.py:6-63
* SO3_Rotation.rotate / rotate_inv / Wigner     so3.py:485-531 (D from the rotation matrix directly,
                                                 e3nn_so3.wigner_from_matrix; pinned to the reference's
                                                 Jd.pt construction by tests/golden/eqv2.npz)
* CoefficientMappingModule (to_m, rescale)      so3.py:30-185
* SO3_Grid (to / from grid matrices)            so3.py:534-642 (e3nn grids: e3nn_so3.ToS2Grid/FromS2Grid)
* SO3_LinearV2                                  so3.py:695-745
* SO2_Convolution / SO2_m_Convolution           so2_ops.py:13-238
* RadialFunction                                radial_function.py:5-32
* EdgeDegreeEmbedding                           input_block.py:11-138
* EquivariantRMSNormArraySphericalHarmonicsV2   layer_norm.py:327-441 (norm_type "rms_norm_sh")
* SO2EquivariantGraphAttention                  transformer_block.py:22-370 (eval: no alpha dropout)
* FeedForwardNetwork (separable S2 activation)  transformer_block.py:373-530
* TransBlockV2 (eval: no drop path)             transformer_block.py:533-728
* SeparableS2Activation / S2Activation /
  SmoothLeakyReLU                               activation.py:62-202
* torch_geometric.utils.softmax                 segment softmax over edge_index[1] (+1e-16)

Supported: lmax_list = [lmax <= 6] (e3nn_so3.LMAX_SUPPORTED), one resolution, use_atom_edge_embedding and not shared,
use_m_share_rad False, distance_function "projection", use_sep_s2_act (the C4 configuration).
``p`` maps the reference state-dict keys to float64 tensors.
"""
from __future__ import annotations

import math

import torch

from . import e3nn_so3 as E

AVG_DEGREE = 23.395238876342773      # equiformer_v2_nbody.py:36


class Layout:
    """Coefficient bookkeeping of CoefficientMappingModule for one (lmax, mmax)."""

    def __init__(self, lmax: int, mmax: int):
        self.lmax, self.mmax = lmax, mmax
        self.full = [(l, m) for l in range(lmax + 1) for m in range(-l, l + 1)]
        self.sel = [i for i, (l, m) in enumerate(self.full) if abs(m) <= mmax]      # coefficient_idx
        self.red = [self.full[i] for i in self.sel]
        perm = []                                                                     # m-primary order
        for m in range(mmax + 1):
            perm += [i for i, (l, mm) in enumerate(self.red) if mm == m]
            if m:
                perm += [i for i, (l, mm) in enumerate(self.red) if mm == -m]
        self.perm = perm
        self.m_size = [lmax - m + 1 for m in range(mmax + 1)]
        # get_rotate_inv_rescale builds its table with torch.ones(...) in the default dtype, so the
        # factor sqrt((2l+1)/(2mmax+1)) is an fp32-rounded constant even in a float64 model
        resc = torch.ones(len(self.full), len(self.full), dtype=torch.float64)
        for l in range(mmax + 1, lmax + 1):
            s = l * l
            resc[s:s + 2 * l + 1, s:s + 2 * l + 1] = float(torch.tensor(math.sqrt((2 * l + 1) / (2 * mmax + 1)),
                                                                        dtype=torch.float32))
        self.rescale = resc[:, self.sel]


def grid_mats(lmax: int, mmax: int):
    """SO3_Grid(lmax, mmax, normalization="component").to_grid_mat / from_grid_mat [b, a, i].
    e3nn builds ToS2Grid / FromS2Grid in the default dtype (float32) and SO3_Grid contracts and
    rescales them in that dtype; a float64 model then holds those float32 values."""
    lat = 2 * (lmax + 1)
    lon = 2 * (mmax + 1) + 1 if lmax == mmax else 2 * mmax + 1
    to = E.ToS2Grid(lmax, (lat, lon), dtype=torch.float32)
    fr = E.FromS2Grid((lat, lon), lmax, dtype=torch.float32)
    tm = torch.einsum("mbi,am->bai", to.shb, to.sha)
    fm = torch.einsum("am,mbi->bai", fr.sha, fr.shb)
    if lmax != mmax:
        for l in range(mmax + 1, lmax + 1):
            s, f = l * l, math.sqrt((2 * l + 1) / (2 * mmax + 1))
            tm[:, :, s:s + 2 * l + 1] = tm[:, :, s:s + 2 * l + 1] * f
            fm[:, :, s:s + 2 * l + 1] = fm[:, :, s:s + 2 * l + 1] * f
    sel = Layout(lmax, mmax).sel
    return tm[:, :, sel].double(), fm[:, :, sel].double()


def silu(x):
    return x * torch.sigmoid(x)


def layer_norm(x, w, b, eps=1e-5):
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * w + b


def linear(p, key, x, bias=True):
    y = x @ p[key + ".weight"].T
    if bias and (key + ".bias") in p:
        y = y + p[key + ".bias"]
    return y


def rad_func(p, key, x):
    """RadialFunction([in, h, h, out]): Linear, LayerNorm, SiLU, Linear, LayerNorm, SiLU, Linear."""
    h = silu(layer_norm(linear(p, key + ".net.0", x), p[key + ".net.1.weight"], p[key + ".net.1.bias"]))
    h = silu(layer_norm(linear(p, key + ".net.3", h), p[key + ".net.4.weight"], p[key + ".net.4.bias"]))
    return linear(p, key + ".net.6", h)


def so3_linear(p, key, x, lmax):
    """SO3_LinearV2: per-degree weight [(lmax+1), out, in], bias on l = 0."""
    lidx = torch.tensor([l for l in range(lmax + 1) for _ in range(2 * l + 1)])
    out = torch.einsum("nmi,moi->nmo", x, p[key + ".weight"][lidx])
    out[:, 0] = out[:, 0] + p[key + ".bias"]
    return out


def rms_norm_sh(p, key, x, lmax, eps=1e-5):
    """EquivariantRMSNormArraySphericalHarmonicsV2 (centering, std_balance_degrees)."""
    x = torch.cat([x[:, :1] - x[:, :1].mean(-1, keepdim=True), x[:, 1:]], 1)
    # balance_degree_weight is a float32 buffer (torch.zeros in the default dtype): 1 / (2l + 1) rounded to
    # float32, then divided by lmax + 1 in float32 (layer_norm.py:370-378), cast with the model
    bal = (torch.tensor([1.0 / (2 * l + 1) for l in range(lmax + 1) for _ in range(2 * l + 1)], dtype=torch.float32)
           / (lmax + 1)).to(x.dtype)
    nrm = torch.einsum("nic,i->nc", x * x, bal).mean(-1)
    s = (nrm + eps) ** -0.5
    lidx = torch.tensor([l for l in range(lmax + 1) for _ in range(2 * l + 1)])
    out = x * s[:, None, None] * p[key + ".affine_weight"][lidx][None]
    out[:, 0] = out[:, 0] + p[key + ".affine_bias"]
    return out


def edge_rot_mat(vec, gauge):
    """init_edge_rot_mat with the random vectors (torch.rand_like draws) supplied as ``gauge``."""
    nx = vec / torch.sqrt((vec ** 2).sum(1)).view(-1, 1)
    v2 = gauge - 0.5
    v2 = v2 / torch.sqrt((v2 ** 2).sum(1)).view(-1, 1)
    v2b = v2.clone()
    v2b[:, 0], v2b[:, 1] = -v2[:, 1], v2[:, 0]
    v2c = v2.clone()
    v2c[:, 1], v2c[:, 2] = -v2[:, 2], v2[:, 1]
    dot = lambda a: (a * nx).sum(1).abs().view(-1, 1)
    v2 = torch.where(dot(v2) > dot(v2b), v2b, v2)
    v2 = torch.where(dot(v2) > dot(v2c), v2c, v2)
    nz = torch.cross(nx, v2, dim=1)
    nz = nz / torch.sqrt((nz ** 2).sum(1, keepdim=True))
    nz = nz / torch.sqrt((nz ** 2).sum(1)).view(-1, 1)
    ny = torch.cross(nx, nz, dim=1)
    ny = ny / torch.sqrt((ny ** 2).sum(1, keepdim=True))
    return torch.stack([nz, nx, -ny], 1)          # rows (z, x, -y) = transpose of [z | x | -y]


def wigner(R, lmax):
    n = (lmax + 1) ** 2
    D = torch.zeros(R.shape[0], n, n, dtype=R.dtype)
    for l in range(lmax + 1):
        D[:, l * l:(l + 1) ** 2, l * l:(l + 1) ** 2] = E.wigner_from_matrix(R, l)
    return D


class Ctx:
    def __init__(self, cfg, p, pos, vel, mass, B, N, gauge):
        self.cfg, self.p = cfg, p
        self.lmax, self.mmax = cfg["lmax_list"][0], cfg["mmax_list"][0]
        assert len(cfg["lmax_list"]) == 1 and self.lmax <= E.LMAX_SUPPORTED
        self.lay = Layout(self.lmax, self.mmax)
        ii, jj = torch.nonzero(~torch.eye(N, dtype=torch.bool), as_tuple=True)     # build_graph_with_knn, k=N-1
        off = torch.arange(0, B * N, N).repeat_interleave(ii.numel())
        self.src, self.dst = ii.repeat(B) + off, jj.repeat(B) + off
        self.Nn = B * N
        self.z = mass.reshape(-1).int().long()
        vec = pos[self.src] - pos[self.dst]
        self.dist = vec.norm(dim=-1)
        self.D = wigner(edge_rot_mat(vec, gauge), self.lmax)
        self.dexp = linear(p, "distance_expansion", self.dist[:, None])
        self.grid_attn = grid_mats(self.lmax, self.mmax)
        self.grid_ffn = grid_mats(self.lmax, self.lmax)

    def x_edge(self, key):
        p = self.p
        return torch.cat([self.dexp, p[key + ".source_embedding.weight"][self.z[self.src]],
                          p[key + ".target_embedding.weight"][self.z[self.dst]]], 1)

    def rotate(self, x):
        return torch.bmm(self.D[:, self.lay.sel, :], x)

    def rotate_inv(self, y):
        Dinv = self.D.transpose(1, 2)[:, :, self.lay.sel] * self.lay.rescale[None]
        return torch.bmm(Dinv, y)

    def to_l_primary(self, xm):
        out = torch.empty_like(xm)
        out[:, self.lay.perm] = xm
        return out

    def so2_conv(self, key, x, x_edge, cout, n_extra=0):
        p, lay = self.p, self.lay
        Ee, _, cin = x.shape
        xm = x[:, lay.perm]
        rad = rad_func(p, key + ".rad_func", x_edge) if x_edge is not None else None
        n0 = lay.m_size[0]
        x0 = xm[:, :n0].reshape(Ee, -1)
        if rad is not None:
            x0 = x0 * rad[:, :n0 * cin]
        y0 = linear(p, key + ".fc_m0", x0)
        extra, y0 = y0[:, :n_extra], y0[:, n_extra:].reshape(Ee, n0, cout)
        outs, off, roff = [y0], n0, n0 * cin
        for m in range(1, lay.mmax + 1):
            nm = lay.m_size[m]
            xm_m = xm[:, off:off + 2 * nm].reshape(Ee, 2, nm * cin)
            if rad is not None:
                xm_m = xm_m * rad[:, None, roff:roff + nm * cin]
            y = linear(p, f"{key}.so2_m_conv.{m - 1}.fc", xm_m, bias=False)
            half = y.shape[-1] // 2
            xr, xi = y[..., :half], y[..., half:]
            ym = torch.stack([xr[:, 0] - xi[:, 1], xr[:, 1] + xi[:, 0]], 1).reshape(Ee, 2 * nm, cout)
            outs.append(ym)
            off, roff = off + 2 * nm, roff + nm * cin
        return self.to_l_primary(torch.cat(outs, 1)), extra

    @staticmethod
    def s2_act(x, grid):
        to, fr = grid
        g = silu(torch.einsum("bai,zic->zbac", to, x))
        return torch.einsum("bai,zbac->zic", fr, g)

    def attention(self, key, x, cout):
        cfg, p = self.cfg, self.p
        nh, na, nv = cfg["num_heads"], cfg["attn_alpha_channels"], cfg["attn_value_channels"]
        x_edge = self.x_edge(key)
        msg = self.rotate(torch.cat([x[self.src], x[self.dst]], 2))
        msg, extra = self.so2_conv(key + ".so2_conv_1", msg, x_edge, cfg["attn_hidden_channels"],
                                   n_extra=nh * na + cfg["attn_hidden_channels"])
        gating, a_in = extra[:, nh * na:], extra[:, :nh * na]
        msg = torch.cat([silu(gating)[:, None], self.s2_act(msg, self.grid_attn)[:, 1:]], 1)
        msg, _ = self.so2_conv(key + ".so2_conv_2", msg, None, nh * nv)
        a = layer_norm(a_in.reshape(-1, nh, na), p[key + ".alpha_norm.weight"], p[key + ".alpha_norm.bias"])
        a = 0.6 * a + 0.4 * a * (2 * torch.sigmoid(a) - 1)                     # SmoothLeakyReLU(0.2)
        logit = torch.einsum("eha,ha->eh", a, p[key + ".alpha_dot"])
        mx = torch.full((self.Nn, nh), -math.inf, dtype=logit.dtype).scatter_reduce(
            0, self.dst[:, None].expand(-1, nh), logit, "amax", include_self=True)
        ex = torch.exp(logit - mx[self.dst])
        den = torch.zeros(self.Nn, nh, dtype=logit.dtype).index_add_(0, self.dst, ex) + 1e-16
        alpha = ex / den[self.dst]
        msg = (msg.reshape(msg.shape[0], msg.shape[1], nh, nv) * alpha[:, None, :, None]).reshape(msg.shape)
        agg = torch.zeros(self.Nn, (self.lmax + 1) ** 2, nh * nv, dtype=msg.dtype).index_add_(
            0, self.dst, self.rotate_inv(msg))
        return so3_linear(p, key + ".proj", agg, self.lmax)

    def ffn(self, key, x):
        p = self.p
        gating = linear(p, key + ".gating_linear", x[:, 0])
        h = so3_linear(p, key + ".so3_linear_1", x, self.lmax)
        h = torch.cat([silu(gating)[:, None], self.s2_act(h, self.grid_ffn)[:, 1:]], 1)
        return so3_linear(p, key + ".so3_linear_2", h, self.lmax)

    def edge_degree(self):
        C = self.cfg["sphere_channels"]
        r = rad_func(self.p, "edge_degree_embedding.rad_func", self.x_edge("edge_degree_embedding"))
        n0 = self.lay.m_size[0]
        xm = torch.zeros(r.shape[0], len(self.lay.red), C, dtype=r.dtype)
        xm[:, :n0] = r.reshape(-1, n0, C)
        y = self.rotate_inv(self.to_l_primary(xm))
        out = torch.zeros(self.Nn, (self.lmax + 1) ** 2, C, dtype=r.dtype).index_add_(0, self.dst, y)
        return out / AVG_DEGREE


def forward(cfg, p, pos, vel, mass, B, N, gauge, acts=None):
    """EquiformerV2_nbody forward on the tuple branch -> [B*N, 6] (delta pos, vel)."""
    pos, vel, mass = (torch.as_tensor(t, dtype=torch.float64) for t in (pos, vel, mass))
    gauge = torch.as_tensor(gauge, dtype=torch.float64)
    ctx = Ctx(cfg, p, pos.reshape(-1, 3), vel.reshape(-1, 3), mass, B, N, gauge)
    C, L = cfg["sphere_channels"], ctx.lmax
    x = torch.zeros(ctx.Nn, (L + 1) ** 2, C, dtype=torch.float64)
    x[:, 0] = p["sphere_embedding.weight"][ctx.z]
    x[:, 1:4] = linear(p, "velocity_embedding", vel.reshape(-1, 3)).reshape(-1, 3, C)
    ed = ctx.edge_degree()
    x = x + ed
    if acts is not None:
        acts["edge_degree"] = ed
    for i in range(cfg["num_layers"]):
        k = f"blocks.{i}"
        y = ctx.attention(k + ".ga", rms_norm_sh(p, k + ".norm_1", x, L), C) + x
        x = ctx.ffn(k + ".ffn", rms_norm_sh(p, k + ".norm_2", y, L)) + y
        if acts is not None:
            acts[f"block{i}"] = x
    x = rms_norm_sh(p, "norm", x, L)
    if acts is not None:
        acts["final_norm"] = x
    pred = ctx.attention("force_block", x, 2)
    return torch.cat([pred[:, 1:4, 0], pred[:, 1:4, 1]], 1)


def rollout(cfg, p, loc0, vel0, mass, steps, gauges):
    """infer_self_feed.py:99-194 tuple branch with target pos_dt+vel: loc += pred[:3], vel = pred[3:].
    loc0/vel0 [B, N, 3], gauges [steps-1, E, 3] -> (loc, vel) [B, steps, N, 3]."""
    B, N, _ = loc0.shape
    L, V = [torch.as_tensor(loc0, dtype=torch.float64)], [torch.as_tensor(vel0, dtype=torch.float64)]
    for s in range(steps - 1):
        pr = forward(cfg, p, L[-1], V[-1], mass, B, N, gauges[s])
        L.append(L[-1] + pr[:, :3].reshape(B, N, 3))
        V.append(pr[:, 3:].reshape(B, N, 3))
    return torch.stack(L, 1), torch.stack(V, 1)
