"""PONITA: host module vs reference (grid, init, state_dict), packed-operand
emulation on CPU, and the HIP path vs the reference golden vectors and the
numpy oracle on the GPU.

Tolerance for the fp32 HIP path (SEGNN's, r03): per output column c,
max |gpu - ref| <= 1e-5 * max |ref[:, c]| + 1e-7 for a forward (vs the reference's golden vectors and
vs the numpy oracle); rollouts 1e-5 * (frame + 1) per column; calibrated weights to 1e-5 relative
(fp32 std()s)."""
import numpy as np
import pytest
import torch
from conftest import assert_cols

import nbody_amd.graph as G
import nbody_amd.ponita as P
from oracle import ponita as op
from oracle.graph import fc_edge_index
from oracle.rollout import ponita_step
from oracle.rollout import rollout as oracle_rollout
from scipy.special import erf


def make(hidden=32, layers=2, dtype=torch.float32, **kw):
    torch.manual_seed(0)
    m = P.PONITA_NBODY(hidden_dim=hidden, layers=layers, lr=1e-3, **kw).to(dtype)
    m.model.materialize()
    return m


def ref_params(g, tag):
    pre = tag + "/param/"
    return {k[len(pre):]: g[k] for k in g.files if k.startswith(pre)}


def load_golden(model, g, tag, device="cpu"):
    sd = {k: torch.from_numpy(np.array(v)) for k, v in ref_params(g, tag).items()}
    model.load_state_dict(sd, strict=True)
    model.model.ori_grid.copy_(torch.from_numpy(g[tag + "/ori_grid"]))
    return model.to(device)


@pytest.mark.parametrize("tag,dtype", [("f32", torch.float32), ("f64", torch.float64)])
def test_grid_and_init_match_reference(golden, tag, dtype):
    """Same RNG consumption as the reference: S2 repulsion grid, Linear inits and
    the lazily materialised basis layers bit-exact; conv kernels differ from the
    fixture only by the one-time calibration factor (a per-tensor constant)."""
    g = golden("ponita")
    m = make(dtype=dtype)
    np.testing.assert_array_equal(m.model.ori_grid.numpy(), g[tag + "/ori_grid"])
    sd = m.state_dict()
    ref = ref_params(g, tag)
    assert set(sd) == set(ref) | {"model.ori_grid"}
    for k, v in ref.items():
        a = sd[k].numpy()
        if k.endswith("conv.kernel.weight") or k.endswith("conv.fiber_kernel.weight"):
            r = v / a
            assert np.ptp(r) <= 1e-6 * np.abs(r).max()
        elif k.endswith("callibrated"):
            assert not a and v
        else:
            np.testing.assert_array_equal(a, v, err_msg=k)


def test_reference_checkpoint_loads_and_keeps_grid(golden):
    g = golden("ponita")
    m = make()
    grid = m.model.ori_grid.clone()
    ref = {k: torch.from_numpy(np.array(v)) for k, v in ref_params(g, "f32").items()}
    m.load_state_dict(ref, strict=True)          # no ori_grid key: constructed grid kept
    assert torch.equal(m.model.ori_grid, grid)
    sd = m.state_dict()
    sd["model.ori_grid"] = torch.zeros_like(grid)
    m.load_state_dict(sd)
    assert torch.count_nonzero(m.model.ori_grid) == 0


def test_native_restrictions_are_loud():
    m = make(hidden=48)
    with pytest.raises(NotImplementedError):
        m._weights("cpu")


def gelu(x):
    return 0.5 * x * (1.0 + erf(x / np.sqrt(2.0)))


def emulate(model, pos, vel, mass, B, N):
    """numpy mirror of csrc/ponita.hip driven by the packed (padded) operands:
    destination-major edge slots, orientation-major fibre rows."""
    Pm = {k: v.double().numpy() for k, v in model.packed_matrices("cpu", torch.float64).items()}
    ori = Pm["ori_grid"]
    O, C = ori.shape[0], model.hidden_dim
    V = B * N
    L = len(model.model.interaction_layers)
    src = np.array([[(d // N) * N + (q if q < d % N else q + 1) for q in range(N - 1)] for d in range(V)])
    rel = pos[src] - pos[:, None, :]                                        # [V, N-1, 3]
    a = np.einsum("vqk,ok->voq", rel, ori)
    b = np.linalg.norm(rel[:, None] - a[..., None] * ori[None, :, None], axis=-1)
    p1 = np.stack([a, b], -1)
    p2 = (p1[..., :, None] * p1[..., None, :]).reshape(p1.shape[:-1] + (4,))
    p3 = (p2[..., :, None] * p1[..., None, :]).reshape(p1.shape[:-1] + (8,))
    P16 = np.concatenate([p1, p2, p3, np.zeros(p1.shape[:-1] + (18,))], -1)  # padded to 32
    kb = gelu(gelu(P16 @ Pm["basis1_t"].T + Pm["basis1_b"]) @ Pm["basis2_t"].T[:C] + Pm["basis2_b"])
    s = ori @ ori.T
    fp = np.zeros((O, O, 32))
    fp[..., 0], fp[..., 1], fp[..., 2] = s, s * s, s * s * s
    fkb = gelu(gelu(fp @ Pm["fbasis1_t"].T + Pm["fbasis1_b"]) @ Pm["fbasis2_t"].T[:C] + Pm["fbasis2_b"])
    Bk = fkb.shape[-1]
    fk = fkb @ Pm["fiber_t"].T[:Bk]                                           # [O, O, L*C]
    x = mass.reshape(V, 1, 1) * Pm["embed_w"][:, 0] + np.einsum("vk,ok->vo", vel, ori)[..., None] * Pm["embed_w"][:, 1]
    ro = 0.0
    nro = 0
    for i in range(L):
        p = f"layers.{i}."
        k = kb @ Pm[p + "kernel_t"].T[:Bk]                                    # [V, O, N-1, C]
        x1 = (k * x[src].transpose(0, 2, 1, 3)).sum(2)
        y = np.einsum("voc,opc->vpc", x1, fk[..., i * C:(i + 1) * C]) / O + Pm[p + "conv_bias"]
        mu = y.mean(-1, keepdims=True)
        var = ((y - mu) ** 2).mean(-1, keepdims=True)
        xn = (y - mu) / np.sqrt(var + 1e-5) * Pm[p + "norm_w"] + Pm[p + "norm_b"]
        h = gelu(xn @ Pm[p + "lin1_t"].T[:C] + Pm[p + "lin1_b"])
        x = x + Pm.get(p + "layer_scale", 1.0) * (h @ Pm[p + "lin2_t"].T[:h.shape[-1]] + Pm[p + "lin2_b"])
        if p + "readout_w" in Pm:
            ro = ro + x @ Pm[p + "readout_w"].T + Pm[p + "readout_b"]
            nro += 1
    return np.einsum("voc,ok->vck", ro / nro, ori).reshape(V, 6) / O


def test_packed_emulation_matches_reference(golden):
    g = golden("ponita")
    m = load_golden(make(dtype=torch.float64), g, "f64")
    got = emulate(m, g["loc"].reshape(-1, 3), g["vel"].reshape(-1, 3), g["mass"].reshape(-1), 4, 5)
    np.testing.assert_allclose(got, g["f64/pred"], rtol=1e-10, atol=1e-12)


# ------------------------------------------------------------------ GPU
class Graph:
    pass


def gpu_graph(pos, vel, mass, B, N, device):
    gr = Graph()
    t = lambda a: torch.tensor(np.asarray(a), dtype=torch.float32, device=device)
    gr.pos = t(pos).reshape(-1, 3)
    gr.vec = t(vel).reshape(-1, 1, 3)
    gr.x = t(mass).reshape(-1, 1)
    gr.edge_index = G.fc_edge_index(B, N, device)
    gr.rel_pos = gr.pos[gr.edge_index[0]] - gr.pos[gr.edge_index[1]]
    return gr


@pytest.mark.gpu
def test_gpu_forward_matches_reference(hip_device, golden):
    g = golden("ponita")
    m = load_golden(make(), g, "f32", hip_device)
    with torch.no_grad():
        out = m(gpu_graph(g["loc"], g["vel"], g["mass"], 4, 5, hip_device)).double().cpu().numpy()
    ref = g["f32/pred"]
    assert_cols(out, ref, label="ponita golden forward vs reference fp32")


@pytest.mark.gpu
def test_gpu_first_forward_calibrates_like_reference(hip_device, golden):
    """Fresh seeded model: the first training-mode forward rescales conv.kernel /
    conv.fiber_kernel exactly as the reference's did when the fixture was made."""
    g = golden("ponita")
    m = make().to(hip_device)
    assert m.training
    with torch.no_grad():
        m(gpu_graph(g["loc"], g["vel"], g["mass"], 4, 5, hip_device))
    sd = m.state_dict()
    for k, v in ref_params(g, "f32").items():
        a = sd[k].cpu().numpy()
        if k.endswith("callibrated"):
            assert bool(a)
        else:
            np.testing.assert_allclose(a, v, rtol=1e-5, atol=1e-7, err_msg=k)
    with torch.no_grad():
        out = m(gpu_graph(g["loc"], g["vel"], g["mass"], 4, 5, hip_device)).double().cpu().numpy()
    ref = g["f32/pred"]
    assert_cols(out, ref, label="ponita calibrated forward vs reference fp32")


@pytest.mark.gpu
def test_gpu_rollout_matches_reference(hip_device, golden):
    g = golden("ponita")
    m = load_golden(make(), g, "f32", hip_device)
    t = lambda a: torch.tensor(a, dtype=torch.float32, device=hip_device)
    tp, tv = m.rollout(t(g["loc"]), t(g["vel"]), t(g["mass"]), 10)
    tp, tv = tp.double().cpu().numpy(), tv.double().cpu().numpy()
    rl, rv = g["f32/roll_loc"], g["f32/roll_vel"]
    for k in range(10):
        tol = 1e-5 * (k + 1)
        assert_cols(tp[:, k], rl[:, k], tol, label=f"ponita golden rollout frame {k} pos")
        assert_cols(tv[:, k], rv[:, k], tol, label=f"ponita golden rollout frame {k} vel")


def oracle_params(model):
    return {k: t.double().cpu().numpy() for k, t in model.state_dict().items()}


@pytest.mark.gpu
@pytest.mark.parametrize("B,N,hidden,layers,num_ori", [(64, 5, 128, 6, 20), (3, 2, 32, 1, 20), (2, 9, 64, 2, 12),
                                                       (1, 20, 32, 2, 24)])
def test_gpu_forward_matches_oracle(hip_device, B, N, hidden, layers, num_ori):
    """C3 architecture (6 x 128, 20 orientations) and edge cases: N = 2 (one edge
    per node), N = 9 (G = 8 slots), N = 20 (19 of 32 slots live)."""
    m = make(hidden, layers, num_ori=num_ori).to(hip_device)
    m.eval()                                    # no calibration: compare the constructed weights
    rng = np.random.default_rng(1)
    pos, vel = rng.standard_normal((B * N, 3)), rng.standard_normal((B * N, 3))
    mass = rng.uniform(0.5, 1.5, (B * N, 1))
    ei = fc_edge_index(B, N)
    ref = op.forward(oracle_params(m), mass, vel[:, None, :], ei, pos[ei[0]] - pos[ei[1]],
                     m.model.ori_grid.double().cpu().numpy(), layers)
    with torch.no_grad():
        out = m(gpu_graph(pos, vel, mass, B, N, hip_device)).double().cpu().numpy()
    assert_cols(out, ref, label="ponita forward vs oracle")


@pytest.mark.gpu
def test_gpu_rollout_matches_oracle(hip_device):
    B, N, T = 16, 5, 6
    m = make(64, 3).to(hip_device)
    m.eval()
    rng = np.random.default_rng(2)
    loc, vel = rng.standard_normal((B, N, 3)), rng.standard_normal((B, N, 3)) * 0.1
    mass = np.ones((B, N, 1))
    params = oracle_params(m)
    grid = m.model.ori_grid.double().cpu().numpy()
    rl, rv = oracle_rollout(ponita_step(params, grid, 3), loc, vel, np.zeros_like(loc), mass, T)
    t = lambda a: torch.tensor(a, dtype=torch.float32, device=hip_device)
    tp, tv = m.rollout(t(loc), t(vel), t(mass), T)
    tp, tv = tp.double().cpu().numpy(), tv.double().cpu().numpy()
    mse = ((tp - rl) ** 2).mean() + ((tv - rv) ** 2).mean()
    assert mse <= 1e-5
    for k in range(T):
        tol = 1e-5 * (k + 1)
        assert_cols(tp[:, k], rl[:, k], tol, label=f"ponita rollout frame {k} pos")


@pytest.mark.gpu
def test_gpu_rollout_equals_repeated_forward(hip_device):
    B, N, T = 8, 5, 4
    m = make(32, 2).to(hip_device)
    m.eval()
    rng = np.random.default_rng(3)
    loc = torch.tensor(rng.standard_normal((B, N, 3)), dtype=torch.float32, device=hip_device)
    vel = torch.tensor(rng.standard_normal((B, N, 3)), dtype=torch.float32, device=hip_device)
    mass = torch.ones(B, N, 1, device=hip_device)
    tp, tv = m.rollout(loc, vel, mass, T)
    p, v = loc.reshape(-1, 3), vel.reshape(-1, 3)
    for k in range(1, T):
        with torch.no_grad():
            out = m(gpu_graph(p.cpu().numpy(), v.cpu().numpy(), mass.cpu().numpy(), B, N, hip_device))
        p, v = p + out[:, :3], out[:, 3:]
        assert torch.equal(tp[:, k].reshape(-1, 3), p)
        assert torch.equal(tv[:, k].reshape(-1, 3), v)


def knn_graph(pos, vel, mass, ei, B, N, device):
    gr = Graph()
    t = lambda a: torch.tensor(np.asarray(a), dtype=torch.float32, device=device)
    gr.pos, gr.vec, gr.x = t(pos).reshape(-1, 3), t(vel).reshape(-1, 1, 3), t(mass).reshape(-1, 1)
    gr.edge_index = torch.as_tensor(np.asarray(ei), dtype=torch.int64, device=device)
    gr.batch = torch.arange(B, device=device).repeat_interleave(N)
    gr.rel_pos = gr.pos[gr.edge_index[0]] - gr.pos[gr.edge_index[1]]
    return gr


@pytest.mark.gpu
@pytest.mark.parametrize("B,N,k,hidden,layers,num_ori", [(8, 5, 1, 32, 2, 12), (8, 5, 2, 64, 2, 20),
                                                         (16, 5, 3, 128, 3, 20), (2, 20, 6, 32, 2, 12)])
def test_gpu_knn_graph_forward_matches_oracle(hip_device, B, N, k, hidden, layers, num_ori):
    """build_graph_with_knn's kNN branch (infer_self_feed.py:137-142 with num_neighbors < N-1):
    FiberBundleConv sums over each node's incoming edges (k = 1 leaves nodes with none)."""
    from oracle.graph import knn_edge_index
    m = make(hidden, layers, num_ori=num_ori).to(hip_device)
    m.eval()
    rng = np.random.default_rng(4)
    pos, vel = rng.standard_normal((B * N, 3)), rng.standard_normal((B * N, 3))
    mass = rng.uniform(0.5, 1.5, (B * N, 1))
    ei = knn_edge_index(pos, B, N, k)
    ref = op.forward(oracle_params(m), mass, vel[:, None, :], ei, pos[ei[0]] - pos[ei[1]],
                     m.model.ori_grid.double().cpu().numpy(), layers)
    with torch.no_grad():
        out = m(knn_graph(pos, vel, mass, ei, B, N, hip_device)).double().cpu().numpy()
    assert_cols(out, ref, label="ponita forward vs oracle")


@pytest.mark.gpu
def test_gpu_fc_graph_in_any_edge_order(hip_device):
    """The fully-connected edge set in another order takes the general-graph path: same result."""
    m = make(32, 2).to(hip_device)
    m.eval()
    B, N = 6, 5
    rng = np.random.default_rng(5)
    pos, vel, mass = rng.standard_normal((B * N, 3)), rng.standard_normal((B * N, 3)), np.ones((B * N, 1))
    with torch.no_grad():
        ref = m(gpu_graph(pos, vel, mass, B, N, hip_device)).double().cpu().numpy()
        ei = fc_edge_index(B, N)[:, np.random.default_rng(6).permutation(B * N * (N - 1))]
        out = m(knn_graph(pos, vel, mass, ei, B, N, hip_device)).double().cpu().numpy()
    np.testing.assert_allclose(out, ref, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [2, 3])
def test_gpu_knn_rollout_matches_oracle(hip_device, k):
    """rollout(num_neighbors=k): each frame's kNN graph rebuilt on the device vs the oracle loop."""
    B, N, T = 16, 5, 5
    m = make(64, 3).to(hip_device)
    m.eval()
    rng = np.random.default_rng(7)
    loc, vel = rng.standard_normal((B, N, 3)), rng.standard_normal((B, N, 3)) * 0.1
    mass = np.ones((B, N, 1))
    params = oracle_params(m)
    grid = m.model.ori_grid.double().cpu().numpy()
    rl, rv = oracle_rollout(ponita_step(params, grid, 3, num_neighbors=k), loc, vel, np.zeros_like(loc), mass, T)
    t = lambda a: torch.tensor(a, dtype=torch.float32, device=hip_device)
    tp, tv = m.rollout(t(loc), t(vel), t(mass), T, num_neighbors=k)
    tp, tv = tp.double().cpu().numpy(), tv.double().cpu().numpy()
    assert ((tp - rl) ** 2).mean() + ((tv - rv) ** 2).mean() <= 1e-5
    for s in range(T):
        tol = 1e-5 * (s + 1)
        assert_cols(tp[:, s], rl[:, s], tol, label=f"ponita rollout step {s} pos")


@pytest.mark.gpu
def test_gpu_knn_rollout_calibrates_on_first_frame(hip_device):
    """A model owing its calibration runs the calibrating forward on the first frame's kNN graph,
    then the kNN rollout: equal to calibrating by hand on that graph and rolling out."""
    B, N, T, k = 8, 5, 4, 2
    rng = np.random.default_rng(8)
    loc = torch.tensor(rng.standard_normal((B, N, 3)), dtype=torch.float32, device=hip_device)
    vel = torch.tensor(rng.standard_normal((B, N, 3)) * 0.1, dtype=torch.float32, device=hip_device)
    mass = torch.ones(B, N, 1, device=hip_device)
    a, b = make(32, 2).to(hip_device), make(32, 2).to(hip_device)
    tp, tv = a.rollout(loc, vel, mass, T, num_neighbors=k)
    ei = G.build_graph_with_knn(loc.reshape(-1, 3), B, N, hip_device, k)
    with torch.no_grad():
        first = b(knn_graph(loc.reshape(-1, 3).cpu().numpy(), vel.reshape(-1, 3).cpu().numpy(),
                            mass.reshape(-1, 1).cpu().numpy(), ei.cpu().numpy(), B, N, hip_device))
    for (ka, va), (kb, vb) in zip(a.state_dict().items(), b.state_dict().items()):
        torch.testing.assert_close(va, vb, msg=ka)
    torch.testing.assert_close(tp[:, 1].reshape(-1, 3), loc.reshape(-1, 3) + first[:, :3])


@pytest.mark.gpu
def test_gpu_c3_full_batch_slices_match_oracle(hip_device):
    """C3 at its full size (hidden 128, 6 layers, 20 orientations, basis 128, B = 4096:
    838 MB kernel-basis buffer, > 2^31-byte row offsets in the edge-slot arrays): forward and
    a 3-frame rollout of the whole batch on the device; PONITA has no cross-system coupling,
    so a 64-system slice from the start, middle and end of the batch is checked against the
    oracle run on those systems alone."""
    B, N, T = 4096, 5, 3
    m = make(128, 6, num_ori=20).to(hip_device)
    m.eval()
    rng = np.random.default_rng(5)
    loc, vel = rng.standard_normal((B, N, 3)), rng.standard_normal((B, N, 3)) * 0.5
    mass = np.ones((B, N, 1))
    with torch.no_grad():
        out = m(gpu_graph(loc, vel, mass, B, N, hip_device)).double().cpu().numpy().reshape(B, N, 6)
    t = lambda a: torch.tensor(a, dtype=torch.float32, device=hip_device)
    tp, tv = m.rollout(t(loc), t(vel), t(mass), T)
    tp, tv = tp.double().cpu().numpy(), tv.double().cpu().numpy()
    params = oracle_params(m)
    grid = m.model.ori_grid.double().cpu().numpy()
    S = 64
    ei = fc_edge_index(S, N)
    for s0 in (0, B // 2 - S // 2, B - S):
        sl = slice(s0, s0 + S)
        p, v = loc[sl].reshape(-1, 3), vel[sl].reshape(-1, 3)
        ref = op.forward(params, mass[sl].reshape(-1, 1), v[:, None, :], ei, p[ei[0]] - p[ei[1]], grid, 6)
        got = out[sl].reshape(-1, 6)
        assert_cols(got, ref, label=f"ponita C3 slice {s0} forward")
        rl, rv = oracle_rollout(ponita_step(params, grid, 6), loc[sl], vel[sl], np.zeros_like(loc[sl]), mass[sl], T)
        for k in range(T):
            tol = 1e-5 * (k + 1)
            assert_cols(tp[sl, k], rl[:, k], tol, label=f"ponita C3 slice {s0} frame {k} pos")
            assert_cols(tv[sl, k], rv[:, k], tol, label=f"ponita C3 slice {s0} frame {k} vel")


def test_ffn_image_layout():
    """The fused ConvNext MLP slabs (include/nbx.h nbx_ponita_layer.ffn_img_x3) decode to linear_1's
    rows, linear_2's columns under the register-order permutation the kernel relies on
    (po_ffn_kernel: image K slot 16 h + 8 m + i <-> hidden unit (i & 3) + 16 m + 8 (i >> 2) + 4 h);
    the three bf16 parts sum back to the fp32 weight within 2^-24 relative."""
    torch.manual_seed(3)
    C, F = 64, 256
    W1, W2 = torch.randn(F, C), torch.randn(C, F)
    img = P.PONITA_NBODY._ffn_image(W1, W2)
    nj, NT, BLK = F // 32, C // 32, 3 * 2 * 64 * 8
    assert img.shape == (nj, 2 * 2 * NT * 1536) and img.dtype == torch.int16
    bf = img.contiguous().view(torch.bfloat16).float().reshape(nj, 2, NT, 3, 2, 64, 8)
    lane = torch.arange(64)
    for j in range(nj):
        for t in range(NT):
            for m in range(2):
                for i in range(8):
                    w1 = bf[j, 0, t, :, m, :, i].sum(0)           # lane (hidden, h), K chunk t
                    k = 32 * t + 16 * (lane >> 5) + 8 * m + i
                    ref1 = W1[32 * j + (lane & 31), k]
                    assert torch.allclose(w1, ref1, rtol=2 ** -22, atol=0)
                    w2 = bf[j, 1, t, :, m, :, i].sum(0)           # lane (out column, h), output tile t
                    hid = 32 * j + (i & 3) + 16 * m + 8 * (i >> 2) + 4 * (lane >> 5)
                    ref2 = W2[32 * t + (lane & 31), hid]
                    assert torch.allclose(w2, ref2, rtol=2 ** -22, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("hidden", [64, 128])
def test_gpu_fused_convnext_matches_two_gemm_path(hip_device, hidden):
    """po_ffn_kernel (ConvNext MLP fused, hidden activation in registers) against the two-GEMM path
    (linear_1 -> HBM -> linear_2) on the same weights: both are fp32-accurate bf16x3 products, so
    they agree to fp32 rounding."""
    B, N = 96, 5
    m = make(hidden, 2, num_ori=12).to(hip_device)
    m.eval()
    rng = np.random.default_rng(21)
    loc, vel = rng.standard_normal((B, N, 3)), rng.standard_normal((B, N, 3)) * 0.5
    mass = np.ones((B, N, 1))
    with torch.no_grad():
        fused = m(gpu_graph(loc, vel, mass, B, N, hip_device)).double().cpu().numpy()
        W = m._weights(hip_device)
        for i in range(W.num_layers):
            assert W.layers[i].ffn_img_x3
            W.layers[i].ffn_img_x3 = None
        plain = m(gpu_graph(loc, vel, mass, B, N, hip_device)).double().cpu().numpy()
    assert np.abs(fused - plain).max() <= 2e-5 * np.abs(plain).max() + 1e-7
