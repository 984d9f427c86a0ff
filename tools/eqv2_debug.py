"""Stage-by-stage comparison of the native EquiformerV2 workspace with the float64 oracle (debug aid).

After one forward the workspace holds the force block's edge buffers; each stage is recomputed in
float64 from the GPU's own inputs to that stage, so the first wrong stage stands out."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
from eqv2_params import param_value  # noqa: E402
from oracle import equiformer_v2 as EQ  # noqa: E402

from nbody_amd.equiformer_v2 import EquiformerV2_nbody  # noqa: E402

STATE = json.load(open(os.path.join(ROOT, "tests", "golden", "eqv2_state.json")))
tag = sys.argv[1] if len(sys.argv) > 1 else "c4"
cfg = STATE[tag]["config"]
dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = EquiformerV2_nbody(**cfg)
with torch.no_grad():
    for k, p in m.named_parameters():
        p.copy_(torch.from_numpy(param_value(k, p.shape)).float())
m = m.to(dev).eval()
P = {k: torch.from_numpy(param_value(k, STATE[tag]["keys"][k])).float().double() for k in STATE[tag]["params"]}

rng = np.random.default_rng(3)
B, N = 2, 6
loc = rng.standard_normal((B, N, 3))
vel = rng.standard_normal((B, N, 3)) * 0.3
mass = np.ones((B, N, 1))
E, V = B * N * (N - 1), B * N
gauge = rng.uniform(0, 1, (E, 3)).astype(np.float32)
t = lambda a: torch.as_tensor(a, dtype=torch.float32, device=dev).reshape(V, -1)
pos = t(loc)
out = m((pos, t(vel), torch.zeros_like(pos), t(mass), pos), torch.arange(B, device=dev).repeat_interleave(N),
        gauge=torch.as_tensor(gauge, device=dev))
torch.cuda.synchronize()
ws = m._ws

C, H, He = cfg["sphere_channels"], cfg["attn_hidden_channels"], cfg["edge_channels"]
nh, na, nv = cfg["num_heads"], cfg["attn_alpha_channels"], cfg["attn_value_channels"]
KV = nh * nv
c32 = lambda x: -(-x // 32) * 32
ld0 = max(c32(nh * na + 4 * H), 3 * C)
ldv0, ldv1 = c32(3 * KV), c32(4 * KV)
off = [0]


def take(n, el=4, dtype=torch.float32):
    off[0] = (off[0] + 255) & ~255
    o = off[0]
    off[0] += n * el
    return ws[o:o + n * el].view(dtype)


bufs = {}
for name, n, dt in [("rot", E * 32, torch.float32), ("zn", V, torch.int32), ("H2", E * He, torch.float32),
                    ("A0", E * 6 * C, torch.float32), ("A1", 2 * E * 4 * C, torch.float32),
                    ("Y0", E * ld0, torch.float32), ("Y1", 2 * E * 4 * H, torch.float32),
                    ("Z0", E * 3 * H, torch.float32), ("Z1", 2 * E * 2 * H, torch.float32),
                    ("L", E * nh, torch.float32), ("V0", E * ldv0, torch.float32), ("V1", 2 * E * ldv1, torch.float32),
                    ("X", V * 9 * C, torch.float32), ("XN", V * 9 * C, torch.float32)]:
    bufs[name] = take(n, 4, dt).cpu().double() if dt == torch.float32 else take(n, 4, dt).cpu()


def rep(name, got, ref):
    got, ref = np.asarray(got, dtype=np.float64), np.asarray(ref, dtype=np.float64)
    err = np.abs(got - ref)
    print(f"{name:10s} max|err| {err.max():.3e}  max|ref| {np.abs(ref).max():.3e}  at {np.unravel_index(err.argmax(), err.shape)}",
          flush=True)


acts = {}
ref_out = EQ.forward(cfg, P, loc, vel, mass, B, N, gauge.astype(np.float64), acts=acts)
rep("out", out.double().cpu().numpy(), ref_out.numpy())
ctx = EQ.Ctx(cfg, P, torch.from_numpy(loc).reshape(-1, 3), torch.from_numpy(vel).reshape(-1, 3), torch.from_numpy(mass),
             B, N, torch.from_numpy(gauge.astype(np.float64)))
rot = bufs["rot"].reshape(E, 32)
rep("R", rot[:, :9].reshape(E, 3, 3), ctx.D[:, 1:4, 1:4])
rep("D2rows", rot[:, 9:24].reshape(E, 3, 5), ctx.D[:, 5:8, 4:9])
rep("dist", rot[:, 24], ctx.dist)
rep("XN", bufs["XN"].reshape(V, 9, C), acts["final_norm"])
# force block stages from the GPU's XN
xn = bufs["XN"].reshape(V, 9, C)
key = "force_block"
x_edge = ctx.x_edge(key)
h = EQ.silu(EQ.layer_norm(EQ.linear(P, key + ".so2_conv_1.rad_func.net.0", x_edge), P[key + ".so2_conv_1.rad_func.net.1.weight"],
                          P[key + ".so2_conv_1.rad_func.net.1.bias"]))
h2 = EQ.silu(EQ.layer_norm(EQ.linear(P, key + ".so2_conv_1.rad_func.net.3", h), P[key + ".so2_conv_1.rad_func.net.4.weight"],
                           P[key + ".so2_conv_1.rad_func.net.4.bias"]))
rep("H2", bufs["H2"].reshape(E, He), h2)
rad = EQ.linear(P, key + ".so2_conv_1.rad_func.net.6", bufs["H2"].reshape(E, He))
msg = ctx.rotate(torch.cat([xn[ctx.src], xn[ctx.dst]], 2))
xm = msg[:, ctx.lay.perm]
A0 = xm[:, :3].reshape(E, -1) * rad[:, :3 * 2 * C]
A1 = xm[:, 3:7].reshape(E, 2, -1) * rad[:, None, 3 * 2 * C:]
rep("A0", bufs["A0"].reshape(E, 6 * C), A0)
rep("A1", bufs["A1"].reshape(2 * E, 4 * C), A1.reshape(2 * E, 4 * C))
Y0 = EQ.linear(P, key + ".so2_conv_1.fc_m0", bufs["A0"].reshape(E, 6 * C))
rep("Y0", bufs["Y0"].reshape(E, ld0)[:, :Y0.shape[1]], Y0)
Y1 = EQ.linear(P, key + ".so2_conv_1.so2_m_conv.0.fc", bufs["A1"].reshape(2 * E, 4 * C), bias=False)
rep("Y1", bufs["Y1"].reshape(2 * E, 4 * H), Y1)
# S2 act from GPU Y0 / Y1
Y0g, Y1g = bufs["Y0"].reshape(E, ld0), bufs["Y1"].reshape(E, 2, 4 * H)
ex = nh * na
m0 = Y0g[:, ex + H:ex + 4 * H].reshape(E, 3, H)
xr, xi = Y1g[..., :2 * H], Y1g[..., 2 * H:]
ym = torch.stack([xr[:, 0] - xi[:, 1], xr[:, 1] + xi[:, 0]], 1).reshape(E, 4, H)
lp = ctx.to_l_primary(torch.cat([m0, ym], 1))
act = torch.cat([EQ.silu(Y0g[:, ex:ex + H])[:, None], ctx.s2_act(lp, ctx.grid_attn)[:, 1:]], 1)
am = act[:, ctx.lay.perm]
rep("Z0", bufs["Z0"].reshape(E, 3 * H), am[:, :3].reshape(E, -1))
rep("Z1", bufs["Z1"].reshape(2 * E, 2 * H), am[:, 3:].reshape(2 * E, 2 * H))
a = EQ.layer_norm(Y0g[:, :ex].reshape(E, nh, na), P[key + ".alpha_norm.weight"], P[key + ".alpha_norm.bias"])
a = 0.6 * a + 0.4 * a * (2 * torch.sigmoid(a) - 1)
rep("L", bufs["L"].reshape(E, nh), torch.einsum("eha,ha->eh", a, P[key + ".alpha_dot"]))
V0 = EQ.linear(P, key + ".so2_conv_2.fc_m0", bufs["Z0"].reshape(E, 3 * H))
rep("V0", bufs["V0"].reshape(E, ldv0)[:, :3 * KV], V0)
V1 = EQ.linear(P, key + ".so2_conv_2.so2_m_conv.0.fc", bufs["Z1"].reshape(2 * E, 2 * H), bias=False)
rep("V1", bufs["V1"].reshape(2 * E, ldv1)[:, :4 * KV], V1)
