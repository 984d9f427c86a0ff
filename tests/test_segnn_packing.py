"""CPU check of the SEGNN kernel decomposition: a numpy emulation of every kernel
in csrc/segnn.hip, fed with the product module's packed operands, must equal the
oracle forward on the same parameters.  (The GPU itself is checked in
test_gpu_segnn.py; this pins the packing formulas and the per-node factorisation
of message_layer_1 without a device.)"""
import numpy as np
import pytest
import torch

import nbody_amd.segnn as S
from oracle.graph import fc_edge_index
from oracle.segnn import SEGNNOracle, o3_transform

C_SILU, C_SIG = 1.6791767923989418, 1.8467055342154763
C1 = S.SH_C1


def silu(x):
    return x / (1 + np.exp(-x))


def sig(x):
    return 1 / (1 + np.exp(-x))


def emulate(model, pos, vel, mass, B, N, training=True, gemm=None):
    """Mirror of forward_impl in csrc/segnn.hip (fp64).  ``gemm(A, key)`` (optional) replaces every
    TP contraction A @ P[key].T, e.g. by an emulation of a reduced-operand MFMA path."""
    P = {k: v.double().numpy() for k, v in model.packed_matrices("cpu", torch.float64).items()}
    if gemm is not None:
        _mm = gemm
    else:
        def _mm(A, key):
            return A @ P[key].T
    sd = {k: v.double().numpy().copy() for k, v in model.state_dict().items()}
    M = model.mul
    V = B * N
    # featurize (dst-major edges)
    d_of = np.repeat(np.arange(V), N - 1)
    q = np.tile(np.arange(N - 1), V)
    dl = d_of % N
    src = (d_of // N) * N + np.where(q < dl, q, q + 1)
    rel = pos[src] - pos[d_of]
    dist = np.sqrt((rel ** 2).sum(1))
    rh = rel / np.maximum(dist, 1e-12)[:, None]
    pm = mass[src] * mass[d_of]
    na = np.zeros((V, 3))
    np.add.at(na, d_of, C1 * rh)
    na = na / max(N - 1, 1) + C1 * vel / np.maximum(np.linalg.norm(vel, axis=1), 1e-12)[:, None]
    u0 = pos - pos.mean(1, keepdims=True)
    vn = np.linalg.norm(vel, axis=1)
    e = P["emb"]
    xs = (u0 * na).sum(1)[:, None] * e[2] + (vel * na).sum(1)[:, None] * e[3] + vn[:, None] * e[4] + P["emb_bias"]
    xv = np.stack([u0[:, k, None] * e[0] + vel[:, k, None] * e[1] + (vn * na[:, k])[:, None] * e[5]
                   for k in range(3)])                                    # [3, V, M]
    for li in range(model.num_layers):
        p = f"layers.{li}."
        nps = _mm(xs, p + "node_pre_s_t")                                # [V, 6M]
        npv = np.stack([_mm(xv[k], p + "node_pre_v_t") for k in range(3)])  # [3, V, 6M]
        amf = np.stack([dist, pm], 1) @ P[p + "msg1_amf"]                 # [E, 3M]
        b1 = P[p + "msg1_bias"]
        sa = nps[d_of, :M] + nps[src, 3 * M:4 * M] + amf[:, :M] + b1[:M]
        sg = nps[d_of, M:2 * M] + nps[src, 4 * M:5 * M] + amf[:, M:2 * M] + b1[M:]
        t = nps[d_of, 2 * M:3 * M] + nps[src, 5 * M:] + amf[:, 2 * M:]
        v = []
        for k in range(3):
            sa = sa + rh[:, k, None] * (npv[k][d_of, :M] + npv[k][src, 3 * M:4 * M])
            sg = sg + rh[:, k, None] * (npv[k][d_of, M:2 * M] + npv[k][src, 4 * M:5 * M])
            v.append(rh[:, k, None] * t + npv[k][d_of, 2 * M:3 * M] + npv[k][src, 5 * M:])
        g = C_SIG * sig(sg)
        m1v = np.stack([g * vk for vk in v])
        m1s = np.concatenate([C_SILU * silu(sa), (m1v * rh.T[:, :, None]).sum(0)], 1)
        g2s = _mm(m1s, p + "msg2_s_t")
        g2v = np.stack([_mm(m1v[k], p + "msg2_v_t") for k in range(3)])
        b2 = P[p + "msg2_bias"]
        ms = C_SILU * silu(g2s[:, :M] + b2[:M])
        gg = C_SIG * sig(g2s[:, M:2 * M] + b2[M:])
        mv = np.stack([gg * (rh[:, k, None] * g2s[:, 2 * M:] + g2v[k]) for k in range(3)])
        E = len(d_of)
        bnw, bnb = sd[p + "message_norm.weight"], sd[p + "message_norm.bias"]
        if training:
            mu = ms.mean(0)
            var = (ms ** 2).mean(0) - mu ** 2
            nv = (mv ** 2).sum(0).sum(0) / (3 * E)
        else:
            mu, var, nv = sd[p + "message_norm.running_mean"], sd[p + "message_norm.running_var"][:M], \
                sd[p + "message_norm.running_var"][M:]
        sc_s, sc_v = bnw[:M] / np.sqrt(var + 1e-5), bnw[M:] / np.sqrt(nv + 1e-5)
        sh = bnb - sc_s * mu
        ags = np.zeros((V, M)); np.add.at(ags, d_of, ms)
        agv = np.zeros((3, V, M))
        for k in range(3):
            np.add.at(agv[k], d_of, mv[k])
        a_s = sc_s * ags + (N - 1) * sh
        a_v = sc_v * agv
        u1s = np.concatenate([xs, a_s, (xv * na.T[:, :, None]).sum(0), (a_v * na.T[:, :, None]).sum(0)], 1)
        g3s = _mm(u1s, p + "upd1_s_t")
        g3v = np.stack([_mm(np.concatenate([xv[k], a_v[k]], 1), p + "upd1_v_t") for k in range(3)])
        b3 = P[p + "upd1_bias"]
        hs = C_SILU * silu(g3s[:, :M] + b3[:M])
        gh = C_SIG * sig(g3s[:, M:2 * M] + b3[M:])
        hv = np.stack([gh * (na[:, k, None] * g3s[:, 2 * M:] + g3v[k]) for k in range(3)])
        g4s = _mm(np.concatenate([hs, (hv * na.T[:, :, None]).sum(0)], 1), p + "upd2_s_t")
        g4v = np.stack([_mm(hv[k], p + "upd2_v_t") for k in range(3)])
        xs = xs + g4s[:, :M] + P[p + "upd2_bias"]
        xv = np.stack([xv[k] + na[:, k, None] * g4s[:, M:] + g4v[k] for k in range(3)])
        fw, fb = sd[p + "feature_norm.weight"], sd[p + "feature_norm.bias"]
        if training:
            mu, var, nv = xs.mean(0), (xs ** 2).mean(0) - xs.mean(0) ** 2, (xv ** 2).sum(0).sum(0) / (3 * V)
        else:
            mu, var, nv = sd[p + "feature_norm.running_mean"], sd[p + "feature_norm.running_var"][:M], \
                sd[p + "feature_norm.running_var"][M:]
        sc_s, sc_v = fw[:M] / np.sqrt(var + 1e-5), fw[M:] / np.sqrt(nv + 1e-5)
        xs = sc_s * xs + (fb - sc_s * mu)
        xv = sc_v * xv
    g = _mm(np.concatenate([xs, (xv * na.T[:, :, None]).sum(0)], 1), "pp1_s_t")
    gv = np.stack([_mm(xv[k], "pp1_v_t") for k in range(3)])
    b = P["pp1_bias"]
    hs = C_SILU * silu(g[:, :M] + b[:M])
    gh = C_SIG * sig(g[:, M:2 * M] + b[M:])
    hv = np.stack([gh * (na[:, k, None] * g[:, 2 * M:] + gv[k]) for k in range(3)])
    W = P["pp2"]
    t0, t1 = hs @ W[0], hs @ W[1]
    out = np.zeros((V, 6))
    for k in range(3):
        out[:, k] = na[:, k] * t0 + hv[k] @ W[2]
        out[:, 3 + k] = na[:, k] * t1 + hv[k] @ W[3]
    return out


def oracle_forward(model, pos, vel, mass, B, N, training=True):
    om = SEGNNOracle(hidden_features=model.hidden_features, num_layers=model.num_layers)
    params = {k: v.double().numpy() for k, v in model.state_dict().items() if "output_mask" not in k}
    ei = fc_edge_index(B, N)
    x, ea, na, amf = o3_transform(pos, vel, mass[:, None], ei)
    out, _ = om.forward(params, x, ei, ea, na, amf, training=training)
    return out


@pytest.mark.parametrize("hidden,layers,B,N,training", [(16, 2, 3, 5, True), (24, 1, 2, 4, True),
                                                         (16, 2, 2, 5, False), (192, 1, 2, 5, True)])
def test_packed_decomposition_matches_oracle(hidden, layers, B, N, training):
    torch.manual_seed(0)
    model = S.SEGNN(hidden_features=hidden, num_layers=layers)
    with torch.no_grad():   # non-trivial BN affine / running stats
        for mod in model.modules():
            if isinstance(mod, S.BatchNorm):
                mod.weight.uniform_(0.5, 1.5)
                mod.bias.uniform_(-0.2, 0.2)
                mod.running_mean.uniform_(-0.1, 0.1)
                mod.running_var.uniform_(0.5, 1.5)
    rng = np.random.default_rng(5)
    V = B * N
    pos, vel = rng.standard_normal((V, 3)), rng.standard_normal((V, 3))
    mass = rng.uniform(0.5, 1.5, V)
    ref = oracle_forward(model, pos, vel, mass, B, N, training)
    got = emulate(model, pos, vel, mass, B, N, training)
    np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-9)


def test_state_dict_layout_matches_oracle():
    torch.manual_seed(0)
    model = S.SEGNN(hidden_features=192, num_layers=6)
    om = SEGNNOracle(hidden_features=192, num_layers=6)
    sd = {k: tuple(v.shape) for k, v in model.state_dict().items() if "output_mask" not in k}
    assert sd == om.param_shapes()
    assert sum(p.numel() for p in model.parameters()) == 1_947_552


def test_bn_mode_switch():
    """SEGNN.bn_mode (SURVEY §8(e) bn_mode={batch,running}): None follows train()/eval() like the
    reference module; "batch" / "running" override it; anything else is rejected."""
    import pytest
    import nbody_amd.segnn as S
    m = S.SEGNN(hidden_features=16, num_layers=1)
    assert m.train()._bn_batch() and not m.eval()._bn_batch()
    m.bn_mode = "batch"
    assert m.eval()._bn_batch()
    m.bn_mode = "running"
    assert not m.train()._bn_batch()
    m.bn_mode = "sync"
    with pytest.raises(ValueError):
        m._bn_batch()


@pytest.mark.parametrize("hidden,layers,dtype", [(32, 2, torch.float32), (192, 6, torch.float32),
                                                  (64, 3, torch.float64)])
def test_train_operands_equal_train_matrices(hidden, layers, dtype):
    """SEGNN.train_operands (one traced gather + one scatter in the backward) equals the
    differentiable train_matrices composition element for element, and gives the same parameter
    gradients for random operand cotangents (C2 widths included; a float64 module too)."""
    import nbody_amd.segnn as S
    torch.manual_seed(0)
    m = S.SEGNN(hidden_features=hidden, num_layers=layers).to(dtype)
    dev = torch.device("cpu")
    A = m.train_matrices(dev)
    B = m.train_operands(dev)
    assert set(A) == set(B)
    for k in A:
        assert torch.equal(A[k], B[k]), k
    g = {k: torch.randn_like(A[k]) for k in A}
    grads = []
    for P in (A, None):
        m.zero_grad()
        P = P if P is not None else m.train_operands(dev)
        sum((P[k] * g[k]).sum() for k in P).backward()
        grads.append({n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None})
    assert set(grads[0]) == set(grads[1])
    for n in grads[0]:
        assert grads[0][n].dtype == grads[1][n].dtype == dtype
        torch.testing.assert_close(grads[0][n], grads[1][n], rtol=1e-6, atol=1e-6)


def _split_gemms(model):
    """GEMM emulations over the module's packed operands: "f32" = fp32 operands, fp32 accumulation
    (the fp32 MFMA path); "h2" = the fp16x2 path (include/nbx.h "fp16x2 images": weights scaled per
    TP by SEGNN.h2_scale and split into fp16 hi + lo, activations split the same way unscaled, the
    three products hi.lo + lo.hi + hi.hi accumulated in fp32)."""
    Pt = model.packed_matrices("cpu", torch.float64)
    P = {k: v.numpy() for k, v in Pt.items()}
    pair = {"node_pre_s_t": "node_pre_v_t", "node_pre_v_t": "node_pre_s_t"}
    def scale(key):
        pre, base = key.rsplit(".", 1) if "." in key else ("", key)
        other = pair.get(base, base[:-4] + ("_v_t" if base.endswith("_s_t") else "_s_t"))
        okey = (pre + "." if pre else "") + other
        return S.SEGNN.h2_scale(Pt[key], Pt[okey])

    def f32(A, key):
        return (A.astype(np.float32) @ P[key].T.astype(np.float32)).astype(np.float64)

    def h2(A, key):
        s = scale(key)
        W = (P[key].T * s).astype(np.float32)
        wh = W.astype(np.float16).astype(np.float32)
        wl = (W - wh).astype(np.float16).astype(np.float32)
        A = A.astype(np.float32)
        ah = A.astype(np.float16).astype(np.float32)
        al = (A - ah).astype(np.float16).astype(np.float32)
        acc = (ah @ wl + al @ wh) + ah @ wh          # fp32 products of fp16 parts are exact
        return acc.astype(np.float64) / s
    return {"f32": f32, "h2": h2}


def test_fp16x2_gemm_path_is_fp32_accurate():
    """The fp16x2 split path (StatSKH2 kernels) on the C2 model (hidden 192, 6 layers, train-mode
    BatchNorm): with every TP contraction emulated on its fp16x2 operands, the forward stays as close
    to the fp64 forward as the same emulation with plain fp32 operands and fp32 accumulation (the
    fp32 MFMA path): max error <= 2x the fp32 path's.  Measured: 1.2x (8.97e-7 vs 7.31e-7; the fp32 accumulation of
    K = 96..384 products dominates the 2^-22 operand representation error of fp16x2)."""
    torch.manual_seed(0)
    model = S.SEGNN(hidden_features=192, num_layers=6)
    rng = np.random.default_rng(3)
    B, N = 8, 5
    V = B * N
    pos, vel = rng.standard_normal((V, 3)) * 1.2, rng.standard_normal((V, 3))
    mass = np.ones(V)
    ref = emulate(model, pos, vel, mass, B, N, True)
    g = _split_gemms(model)
    e = {k: np.abs(emulate(model, pos, vel, mass, B, N, True, gemm=f) - ref).max() / np.abs(ref).max()
         for k, f in g.items()}
    print(f"C2 forward, max error / output scale vs fp64: fp32 path {e['f32']:.2e}, fp16x2 path {e['h2']:.2e}")
    assert e["h2"] <= 2.0 * e["f32"] and e["h2"] < 1e-5, e
