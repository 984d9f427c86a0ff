"""EGNN-MC: host module vs reference (init, state_dict), packed-operand emulation
on CPU, and the HIP path vs the reference golden vectors on the GPU.
Tolerance for the fp32 HIP path (SEGNN's, r03): per output column c,
max |gpu - ref| <= 1e-5 * max |ref[:, c]| + 1e-7 per forward; rollouts 1e-5 * (frame + 1) per column."""
import numpy as np
import pytest
import torch
from conftest import assert_cols

import nbody_amd.egnn_mc as E
import nbody_amd.graph as G
from oracle import egnn_mc as oe
from oracle.graph import fc_edge_index


def make(hidden=32, layers=2, dtype=torch.float64):
    torch.manual_seed(0)
    return E.EGNNMultiChannel(node_input_dim=2, edge_attr_dim=4, hidden_node_dim=hidden, hidden_edge_dim=hidden,
                              hidden_coord_dim=hidden, num_layers=layers, target_names=("pos_dt", "vel"),
                              activation="silu", coords_weight=1.0, recurrent=True, norm_diff=True,
                              tanh=True).to(dtype)


def test_init_and_state_dict_match_reference(golden):
    g = golden("egnn_mc")
    ref = {k[len("f64/param/"):]: g[k] for k in g.files if k.startswith("f64/param/")}
    sd = make().state_dict()
    assert set(sd) == set(ref)
    for k, v in ref.items():
        np.testing.assert_array_equal(sd[k].numpy(), v)


def emulate(model, pos, vel, mass, B, N):
    """numpy mirror of csrc/egnn.hip driven by the packed (padded) operands."""
    P = {k: v.double().numpy() for k, v in model.packed_matrices("cpu", torch.float64).items()}
    H = model.hidden_node_dim
    kp = (H + 31) // 32 * 32
    silu = lambda x: x / (1 + np.exp(-x))
    ei = fc_edge_index(B, N)
    row, col = ei
    V = B * N
    x4 = np.zeros((V, 32)); x4[:, 0] = np.linalg.norm(vel, axis=1); x4[:, 1] = mass
    d = pos[row] - pos[col]
    d2 = (d ** 2).sum(1)
    dh = d / np.maximum(np.sqrt(d2), 1e-12)[:, None]
    ea = np.stack([mass[row] * mass[col], (vel[row] * dh).sum(1), (vel[col] * dh).sum(1), d2], 1)
    h = x4 @ P["emb_t"].T + P["emb_b"]
    coord = pos.copy()
    pad = lambda a, w: np.pad(a, ((0, 0), (0, w - a.shape[1])))
    for i in range(model.num_layers):
        p = f"layers.{i}."
        diff = coord[row] - coord[col]
        rad = (diff ** 2).sum(1, keepdims=True)
        diff = diff / np.maximum(np.sqrt(rad), 1.0)
        a = np.concatenate([pad(h[row], kp), pad(h[col], kp), pad(np.concatenate([rad, ea], 1), 32)], 1)
        ef = silu(silu(a @ P[p + "e0_t"].T + P[p + "e0_b"]) @ P[p + "e1_t"].T + P[p + "e1_b"])
        c = np.tanh(silu(ef @ P[p + "c0_t"].T + P[p + "c0_b"]) @ P[p + "c1_w"])
        trans = np.clip(diff * c[:, None], -100, 100).reshape(V, N - 1, 3).mean(1)
        cv = silu(h @ P[p + "v0_t"].T + P[p + "v0_b"]) @ P[p + "v1_w"] + P[p + "v1_b"]
        agg = ef.reshape(V, N - 1, H).mean(1)
        nh = silu(np.concatenate([pad(h, kp), pad(agg, kp)], 1) @ P[p + "n0_t"].T + P[p + "n0_b"])
        h = h + nh @ P[p + "n1_t"].T + P[p + "n1_b"]
        coord = coord + trans + cv[:, None] * vel
    hin = np.concatenate([pad(h, kp), pad(np.concatenate([coord - pos, vel], 1), 32)], 1)
    outs = []
    for t in range(2):
        p = f"heads.{t}."
        y = silu(silu(hin @ P[p + "w0_t"].T + P[p + "b0"]) @ P[p + "w1_t"].T + P[p + "b1"])
        outs.append(y @ P[p + "w2_t"].T + P[p + "b2"])
    return np.concatenate(outs, 1)


def test_packed_emulation_matches_reference(golden):
    g = golden("egnn_mc")
    model = make()
    loc, vel, mass = g["loc"].reshape(-1, 3), g["vel"].reshape(-1, 3), g["mass"].reshape(-1)
    got = emulate(model, loc, vel, mass, 4, 5)
    np.testing.assert_allclose(got, g["f64/pred"], rtol=1e-10, atol=1e-12)


class Graph:
    pass


@pytest.mark.gpu
def test_gpu_forward_matches_reference(hip_device, golden):
    g = golden("egnn_mc")
    model = make(dtype=torch.float32).to(hip_device)
    gr = Graph()
    gr.pos = torch.tensor(g["loc"].reshape(-1, 3), dtype=torch.float32, device=hip_device)
    gr.vel = torch.tensor(g["vel"].reshape(-1, 3), dtype=torch.float32, device=hip_device)
    gr.mass = torch.tensor(g["mass"].reshape(-1, 1), dtype=torch.float32, device=hip_device)
    gr.edge_index = G.fc_edge_index(4, 5, hip_device)
    with torch.no_grad():   # the inference kernel (grad mode runs the training forward, tested below)
        out = model(gr).double().cpu().numpy()
    ref = g["f64/pred"]
    assert_cols(out, ref, label="egnn_mc forward")


@pytest.mark.gpu
def test_gpu_rollout_matches_reference(hip_device, golden):
    g = golden("egnn_mc")
    model = make(dtype=torch.float32).to(hip_device)
    t = lambda a: torch.tensor(a, dtype=torch.float32, device=hip_device)
    tp, tv = model.rollout(t(g["loc"]), t(g["vel"]), t(g["mass"]), 10)
    tp, tv = tp.double().cpu().numpy(), tv.double().cpu().numpy()
    rl, rv = g["f64/roll_loc"], g["f64/roll_vel"]
    for k in range(10):
        tol = 1e-5 * (k + 1)
        assert_cols(tp[:, k], rl[:, k], tol, label=f"egnn_mc golden rollout frame {k} pos")
        assert_cols(tv[:, k], rv[:, k], tol, label=f"egnn_mc golden rollout frame {k} vel")


@pytest.mark.gpu
@pytest.mark.parametrize("B,N,hidden,layers", [(64, 5, 128, 6), (3, 7, 64, 2), (2, 2, 32, 1)])
def test_gpu_forward_matches_oracle(hip_device, B, N, hidden, layers):
    """C1 shape (B=64, 6 x 128) and edge cases vs the numpy oracle."""
    model = make(hidden, layers, torch.float32).to(hip_device)
    params = {k: v.double().cpu().numpy() for k, v in model.state_dict().items()}
    rng = np.random.default_rng(1)
    pos, vel = rng.standard_normal((B * N, 3)), rng.standard_normal((B * N, 3))
    mass = np.ones((B * N, 1))
    ei = fc_edge_index(B, N)
    x, ea = oe.preprocess(pos, vel, mass, ei)
    ref = oe.forward(params, x, pos, vel, ei, ea, layers)
    gr = Graph()
    gr.pos = torch.tensor(pos, dtype=torch.float32, device=hip_device)
    gr.vel = torch.tensor(vel, dtype=torch.float32, device=hip_device)
    gr.mass = torch.tensor(mass, dtype=torch.float32, device=hip_device)
    gr.edge_index = G.fc_edge_index(B, N, hip_device)
    with torch.no_grad():
        out = model(gr).double().cpu().numpy()
    assert_cols(out, ref, label="egnn_mc forward vs oracle")


# ------------------------------------------------------------------ training step (csrc/egnn_train.hip)
def _grad_model(Z, tag, device):
    H = Z[f"{tag}/param/embedding.weight"].shape[0]
    L = len({k.split(".")[1] for k in Z.files if k.startswith(f"{tag}/param/layers.")})
    model = make(H, L, torch.float32).to(device)
    with torch.no_grad():
        for k, p in model.named_parameters():
            p.copy_(torch.from_numpy(Z[f"{tag}/param/{k}"]).float())
    return model


def _grad_graph(Z, tag, device):
    gr = Graph()
    B, N = Z[f"{tag}/loc"].shape[:2]
    t = lambda a, w: torch.tensor(a.reshape(-1, w), dtype=torch.float32, device=device)
    gr.pos, gr.vel, gr.mass = t(Z[f"{tag}/loc"], 3), t(Z[f"{tag}/vel"], 3), t(Z[f"{tag}/mass"], 1)
    gr.edge_index = G.fc_edge_index(B, N, device)
    return gr


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["h32", "h64"])
def test_gpu_training_gradients_match_reference(hip_device, golden, tag):
    """loss = sum(pred * G): every parameter gradient of the native backward against the reference
    module's float64 autograd (tests/golden/egnn_mc_grad.npz, make_golden.py --only egnn_grad).
    Tolerance per tensor: |g - ref| <= 2e-4 max|ref| + 1e-7 (fp32 forward + backward)."""
    Z = golden("egnn_mc_grad")
    model = _grad_model(Z, tag, hip_device)
    pred = model(_grad_graph(Z, tag, hip_device))
    assert pred.grad_fn is not None
    ref = Z[f"{tag}/pred"]
    got = pred.detach().double().cpu().numpy()
    assert_cols(got, ref, label="egnn_mc training forward")
    (pred * torch.tensor(Z[f"{tag}/G"], dtype=torch.float32, device=hip_device)).sum().backward()
    for k, p in model.named_parameters():
        r = Z[f"{tag}/grad/{k}"]
        g = p.grad.double().cpu().numpy()
        assert np.abs(g - r).max() <= 2e-4 * np.abs(r).max() + 1e-7, (k, np.abs(g - r).max(), np.abs(r).max())


@pytest.mark.gpu
def test_gpu_training_step_c1_shape(hip_device):
    """C1 widths (6 x 128, B = 64, N = 5): an optimizer step through the reference trainer's calls
    (zero_grad, forward, MSE loss, backward, clip, step) runs on the native path, the gradient is
    finite and equals the sum of two half-batch gradients (systems are independent)."""
    torch.manual_seed(0)
    model = make(128, 6, torch.float32).to(hip_device)
    rng = np.random.default_rng(3)
    B, N = 64, 5
    pos, vel = rng.standard_normal((B * N, 3)), rng.standard_normal((B * N, 3)) * 0.5
    tgt = torch.tensor(rng.standard_normal((B * N, 6)) * 0.1, dtype=torch.float32, device=hip_device)

    def graph(lo, hi):
        gr = Graph()
        gr.pos = torch.tensor(pos[lo * N:hi * N], dtype=torch.float32, device=hip_device)
        gr.vel = torch.tensor(vel[lo * N:hi * N], dtype=torch.float32, device=hip_device)
        gr.mass = torch.ones(gr.pos.shape[0], 1, device=hip_device)
        gr.edge_index = G.fc_edge_index(hi - lo, N, hip_device)
        return gr

    def grads(lo, hi):
        model.zero_grad()
        loss = ((model(graph(lo, hi)) - tgt[lo * N:hi * N]) ** 2).sum()
        loss.backward()
        return [p.grad.clone() for p in model.parameters()]

    full, a, b = grads(0, B), grads(0, B // 2), grads(B // 2, B)
    for f, x, y in zip(full, a, b):
        assert torch.isfinite(f).all()
        assert torch.allclose(f, x + y, rtol=1e-4, atol=1e-6 * f.abs().max().item())
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    before = [p.detach().clone() for p in model.parameters()]
    opt.zero_grad()
    loss = torch.nn.functional.mse_loss(model(graph(0, B)), tgt)
    loss.backward()
    torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
    opt.step()
    assert any(not torch.equal(p0, p1) for p0, p1 in zip(before, model.parameters()))


@pytest.mark.gpu
def test_gpu_training_step_hip_graph_matches_eager(hip_device):
    """bench.py's training line replays the whole step (forward, backward, clip, fused AdamW with
    a device-resident lr) as one HIP graph; twelve graph-path steps (three eager warm-up steps on a
    side stream, then nine back-to-back replays) land on the same weights as twelve eager steps."""
    B, N, K, W = 16, 5, 12, 3
    rng = np.random.default_rng(5)
    gr = Graph()
    gr.pos = torch.tensor(rng.standard_normal((B * N, 3)), dtype=torch.float32, device=hip_device)
    gr.vel = torch.tensor(rng.standard_normal((B * N, 3)) * 0.5, dtype=torch.float32, device=hip_device)
    gr.mass = torch.ones(B * N, 1, device=hip_device)
    gr.edge_index = G.fc_edge_index(B, N, hip_device)
    gr.nbx_system_size = N  # skips the host-side edge_index check, which cannot run under capture
    tgt = torch.tensor(rng.standard_normal((B * N, 6)) * 0.1, dtype=torch.float32, device=hip_device)

    def run(graph):
        torch.manual_seed(0)
        model = make(64, 4, torch.float32).to(hip_device)
        params = list(model.parameters())
        opt = torch.optim.AdamW(params, lr=1e-3, fused=True, capturable=graph)
        if graph:
            for grp in opt.param_groups:
                grp["lr"] = torch.tensor(1e-3, dtype=torch.float32, device=hip_device)

        def body():
            opt.zero_grad(set_to_none=True)
            loss = torch.nn.functional.mse_loss(model(gr), tgt)
            loss.backward()
            torch.nn.utils.clip_grad_norm_(params, 1.0, foreach=True)
            opt.step()
            return loss

        if not graph:
            for _ in range(K):
                body()
            return params, model
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(W):
                body()
        torch.cuda.current_stream().wait_stream(side)
        cg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(cg):
            body()
        with torch.no_grad():
            model(gr)              # packs the inference weights at their current (pre-replay) values
        for _ in range(K - W):
            cg.replay()
        torch.cuda.synchronize()
        model.invalidate_weights()   # replays update the parameters without bumping _version
        return params, model

    (pe_all, me), (pg_all, mg) = run(False), run(True)
    for pe, pg in zip(pe_all, pg_all):
        assert torch.allclose(pe, pg, rtol=1e-5, atol=1e-6), (pe - pg).abs().max().item()
    # a no-grad (inference) forward after the replays sees the replayed weights
    with torch.no_grad():
        oe_, og_ = me(gr), mg(gr)
    assert torch.allclose(oe_, og_, rtol=1e-4, atol=1e-5), (oe_ - og_).abs().max().item()



def test_training_blob_index_map():
    """The training step packs the persist blob with one scatter of the flattened parameters and
    maps the blob gradient back with one gather (EGNNMultiChannel._train_layout): the scatter must
    reproduce persist_blob exactly and the gather must be its adjoint (every parameter element read
    from its own blob slot, the padding never)."""
    torch.manual_seed(3)
    m = make(hidden=32, layers=2, dtype=torch.float32)
    params, idx, nblob = m._train_layout("cpu")
    flat = torch.cat([q.detach().reshape(-1) for q in params])
    blob = torch.zeros(nblob).index_copy_(0, idx, flat)
    torch.testing.assert_close(blob, m.persist_blob("cpu"), rtol=0, atol=0)
    assert idx.unique().numel() == idx.numel() == sum(q.numel() for q in m.parameters())
    g = torch.randn(nblob)
    ref = torch.autograd.grad(m.persist_blob("cpu", differentiable=True), params, g)
    got = g.index_select(0, idx)
    torch.testing.assert_close(got, torch.cat([r.reshape(-1) for r in ref]), rtol=0, atol=0)


@pytest.mark.parametrize("tag", ["h32", "h64"])
def test_torch_restatement_matches_reference_gradients(golden, tag):
    """oracle/egnn_mc_torch.py (the CPU baseline of bench.py --model egnn_mc_train) reproduces the
    reference's float64 prediction and parameter gradients."""
    from oracle import egnn_mc_torch as OT
    Z = golden("egnn_mc_grad")
    P = {k[len(f"{tag}/param/"):]: torch.from_numpy(Z[k]).clone().requires_grad_(True)
         for k in Z.files if k.startswith(f"{tag}/param/")}
    B, N = Z[f"{tag}/loc"].shape[:2]
    L = len({k.split(".")[1] for k in P if k.startswith("layers.")})
    t = lambda a, w: torch.from_numpy(a.reshape(-1, w))
    pred = OT.forward(P, t(Z[f"{tag}/loc"], 3), t(Z[f"{tag}/vel"], 3), t(Z[f"{tag}/mass"], 1), B, N, L)
    np.testing.assert_allclose(pred.detach().numpy(), Z[f"{tag}/pred"], rtol=1e-10, atol=1e-12)
    (pred * torch.from_numpy(Z[f"{tag}/G"])).sum().backward()
    for k, p in P.items():
        np.testing.assert_allclose(p.grad.numpy(), Z[f"{tag}/grad/{k}"], rtol=1e-9, atol=1e-12, err_msg=k)


# ------------------------------------------------------------------ kNN graphs
def test_knn_table_layout():
    """The module turns build_graph_with_knn's kNN graph into the kernel's [B N][k] local neighbour
    table, and refuses graphs without k edges at every row node (CPU, host logic only)."""
    from oracle.graph import knn_edge_index
    rng = np.random.default_rng(2)
    B, N, k = 3, 6, 2
    loc = rng.standard_normal((B * N, 3))
    ei = torch.from_numpy(knn_edge_index(loc, B, N, k))
    kk, nbr = E.EGNNMultiChannel._knn_table(ei, B, N, "cpu")
    assert kk == k and nbr.dtype == torch.int32 and nbr.shape == (B * N * k,)
    np.testing.assert_array_equal(nbr.numpy(), ei[1].numpy() % N)
    with pytest.raises(NotImplementedError):   # ragged: drop one edge
        E.EGNNMultiChannel._knn_table(ei[:, 1:], B, N, "cpu")
    with pytest.raises(NotImplementedError):   # not grouped by row
        E.EGNNMultiChannel._knn_table(ei.flip(0), B, N, "cpu")


def _knn_graph(pos, vel, mass, B, N, k, device):
    from oracle.graph import knn_edge_index
    gr = Graph()
    gr.pos = torch.tensor(pos, dtype=torch.float32, device=device)
    gr.vel = torch.tensor(vel, dtype=torch.float32, device=device)
    gr.mass = torch.tensor(mass, dtype=torch.float32, device=device)
    gr.edge_index = torch.from_numpy(knn_edge_index(pos.astype(np.float32).astype(np.float64), B, N, k)).to(device)
    gr.batch = torch.arange(B, device=device).repeat_interleave(N)
    return gr


@pytest.mark.gpu
@pytest.mark.parametrize("B,N,k,hidden,layers", [(64, 5, 2, 128, 6), (7, 8, 3, 64, 2), (5, 3, 1, 32, 1)])
def test_gpu_forward_knn_matches_oracle(hip_device, B, N, k, hidden, layers):
    """A forward on build_graph_with_knn's graph (the egnn_mc dataloader's num_neighbors < N-1)
    against the numpy oracle on the same edge_index (segment means over k edges per row node)."""
    from oracle.graph import knn_edge_index
    model = make(hidden, layers, torch.float32).to(hip_device)
    params = {kk: v.double().cpu().numpy() for kk, v in model.state_dict().items()}
    rng = np.random.default_rng(4)
    pos, vel = rng.standard_normal((B * N, 3)), rng.standard_normal((B * N, 3))
    mass = rng.uniform(0.5, 2.0, (B * N, 1))
    gr = _knn_graph(pos, vel, mass, B, N, k, hip_device)
    ei = gr.edge_index.cpu().numpy()
    p32 = pos.astype(np.float32).astype(np.float64)
    v32 = vel.astype(np.float32).astype(np.float64)
    m32 = mass.astype(np.float32).astype(np.float64)
    x, ea = oe.preprocess(p32, v32, m32, ei)
    ref = oe.forward(params, x, p32, v32, ei, ea, layers)
    with torch.no_grad():
        out = model(gr).double().cpu().numpy()
    assert_cols(out, ref, label="egnn_mc forward vs oracle")


@pytest.mark.gpu
def test_gpu_rollout_knn_equals_repeated_oracle_forward(hip_device):
    """rollout(num_neighbors=k) rebuilds each frame's kNN graph inside the kernel: frame by frame it
    matches the oracle forward on the oracle's kNN graph of the rollout's own previous frame (the
    per-frame comparison keeps a near-tie in the selection from compounding)."""
    from oracle.graph import knn_edge_index
    B, N, k, T = 32, 6, 3, 6
    model = make(64, 3, torch.float32).to(hip_device)
    params = {kk: v.double().cpu().numpy() for kk, v in model.state_dict().items()}
    rng = np.random.default_rng(6)
    loc, vel = rng.standard_normal((B, N, 3)), rng.standard_normal((B, N, 3)) * 0.3
    mass = np.ones((B, N, 1))
    t = lambda a: torch.tensor(a, dtype=torch.float32, device=hip_device)
    tp, tv = model.rollout(t(loc), t(vel), t(mass), T, num_neighbors=k)
    tp, tv = tp.double().cpu().numpy(), tv.double().cpu().numpy()
    assert np.isfinite(tp).all()
    for f in range(1, T):
        p, v = tp[:, f - 1].reshape(-1, 3), tv[:, f - 1].reshape(-1, 3)
        ei = knn_edge_index(p, B, N, k)
        x, ea = oe.preprocess(p, v, mass.reshape(-1, 1), ei)
        pred = oe.forward(params, x, p, v, ei, ea, 3)
        want_p, want_v = p + pred[:, :3], pred[:, 3:]
        assert np.abs(tp[:, f].reshape(-1, 3) - want_p).max() <= 2e-4 * np.abs(want_p).max() + 1e-5
        assert np.abs(tv[:, f].reshape(-1, 3) - want_v).max() <= 2e-4 * np.abs(want_v).max() + 1e-5


def test_grad_mode_forward_refuses_uncovered_training_inputs():
    """A grad-mode forward the native training step does not cover raises NotImplementedError with
    the reason: a kNN graph (the egnn_mc dataloader's num_neighbors < N-1) and N = 9
    bodies (the step holds a system's activations in LDS for 2 <= N <= 8).  Before, such a forward
    returned the inference result without an autograd graph, so every parameter's .grad stayed None
    and AdamW skipped them silently.  Host logic only: the refusal comes before any device call."""
    from oracle.graph import knn_edge_index
    model = make(32, 2, torch.float32)
    rng = np.random.default_rng(3)
    B, N, k = 2, 6, 2
    pos, vel = rng.standard_normal((B * N, 3)), rng.standard_normal((B * N, 3))
    g = Graph()
    g.pos, g.vel = torch.tensor(pos, dtype=torch.float32), torch.tensor(vel, dtype=torch.float32)
    g.mass = torch.ones(B * N, 1)
    g.edge_index = torch.from_numpy(knn_edge_index(pos, B, N, k))
    g.batch = torch.arange(B).repeat_interleave(N)
    with pytest.raises(NotImplementedError, match="kNN"):
        model(g)
    N = 9
    g.pos, g.vel = torch.zeros(B * N, 3), torch.ones(B * N, 3)
    g.mass = torch.ones(B * N, 1)
    g.edge_index = torch.from_numpy(__import__("oracle.graph", fromlist=["x"]).fc_edge_index(B, N))
    g.batch = torch.arange(B).repeat_interleave(N)
    g.nbx_system_size = N          # (fully connected: skips the device-side edge_index comparison)
    with pytest.raises(NotImplementedError, match="N = 9"):
        model(g)
