"""run_inference on the device for every native family at the reference's default
precision (precision_mode: double, config.yaml:92,177; infer_self_feed.py:45-48), the
absolute-position targets (infer_self_feed.py:185-186), and checkpoint-driven rollouts
(model=None, utils/nbody_utils.py:1316-1407)."""
import numpy as np
import pytest
import torch

import nbody_amd.dataset as D
import nbody_amd.graph as G
import nbody_amd.inference as I
from nbody_amd.egnn_mc import EGNNMultiChannel
from nbody_amd.ponita import PONITA_NBODY
from nbody_amd.segnn import SEGNN

pytestmark = pytest.mark.gpu


class Graph:
    pass


def small_model(kind, device):
    torch.manual_seed(0)
    if kind == "segnn":
        return SEGNN(hidden_features=32, num_layers=2).to(device).train()
    if kind == "ponita":
        return PONITA_NBODY(hidden_dim=32, layers=2, num_ori=8, basis_dim=32).to(device).train()
    return EGNNMultiChannel(node_input_dim=2, edge_attr_dim=4, hidden_node_dim=32, hidden_edge_dim=32,
                            hidden_coord_dim=32, num_layers=2, target_names=("pos_dt", "vel"), norm_diff=True,
                            tanh=True, device=device)


def dataset(device, tmp_path, double=True, target="pos_dt+vel", B=4):
    return D.GravityDatasetOtf(batch_size=B, sim_length=80, num_nodes=5, device=device, double_precision=double,
                               target=target, data_path=str(tmp_path / "sims"), cache_data=False)


def step_forward(model, kind, l, v, m, B, N, device):
    g = Graph()
    g.pos, g.vel, g.mass, g.edge_index = l, v, m, G.fc_edge_index(B, N, device)
    if kind == "ponita":
        g.x, g.vec = m, v.reshape(-1, 1, 3)
    with torch.no_grad():   # the rollout's inference forward (grad mode would run EGNN-MC's training forward)
        return model(g)


@pytest.mark.parametrize("kind", ["segnn", "ponita", "egnn_mc"])
def test_run_inference_default_double_precision(hip_device, tmp_path, kind):
    """The reference default (double) casts the model with .double(); the native path still
    computes in fp32 and returns fp64 arrays.  SEGNN's fp64 BatchNorm buffers are updated
    through fp32 device shadows."""
    ds = dataset(hip_device, tmp_path, double=True)
    model = small_model(kind, hip_device)
    ref = small_model(kind, hip_device)             # fp32 twin: the same weights
    out_dir, locs, vels = I.run_inference(kind, None, model=model, dataset=ds, save_dir=str(tmp_path / "o"),
                                          device=hip_device, max_rollout_steps=5, print_step=False)
    assert locs.dtype == np.float64 and locs.shape == (2, 4, 5, 5, 3)
    assert np.isfinite(locs).all() and np.isfinite(vels).all()
    assert next(model.parameters()).dtype == torch.float64
    loc0 = torch.tensor(locs[0][:, 0], dtype=torch.float32, device=hip_device)
    vel0 = torch.tensor(vels[0][:, 0], dtype=torch.float32, device=hip_device)
    tp, tv = ref.rollout(loc0, vel0, torch.ones(4, 5, 1, device=hip_device), 5)
    np.testing.assert_allclose(locs[1], tp.double().cpu().numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(vels[1], tv.double().cpu().numpy(), rtol=1e-5, atol=1e-5)
    if kind == "segnn":   # fp64 running stats written back, equal to the fp32 twin's
        sd, sr = model.state_dict(), ref.state_dict()
        for k in sd:
            if "running" in k:
                assert sd[k].dtype == torch.float64
                np.testing.assert_allclose(sd[k].cpu().numpy(), sr[k].double().cpu().numpy(), rtol=1e-5, atol=1e-7)
                init = 0.0 if k.endswith("running_mean") else 1.0
                assert (sd[k] != init).any()          # the rollout did update them


@pytest.mark.parametrize("kind", ["segnn", "ponita", "egnn_mc"])
def test_rollout_absolute_target(hip_device, kind):
    """target "pos+vel" (any target but "pos_dt+vel"): pos = pred[:, :3] each step."""
    B, N, T = 3, 5, 4
    model = small_model(kind, hip_device)
    if kind == "ponita":
        model.eval()   # no calibration: the rollout and the forwards see the same weights
        model.model.materialize()
    rng = np.random.default_rng(1)
    loc = torch.tensor(rng.standard_normal((B, N, 3)), dtype=torch.float32, device=hip_device)
    vel = torch.tensor(rng.standard_normal((B, N, 3)), dtype=torch.float32, device=hip_device)
    mass = torch.ones(B, N, 1, device=hip_device)
    sd0 = {k: v.clone() for k, v in model.state_dict().items()}
    tp, tv = model.rollout(loc, vel, mass, T, absolute=True)
    model.load_state_dict(sd0)
    l, v = loc.reshape(-1, 3).clone(), vel.reshape(-1, 3).clone()
    for t in range(1, T):
        out = step_forward(model, kind, l, v, mass.reshape(-1, 1), B, N, hip_device)
        l, v = out[:, :3].contiguous(), out[:, 3:].contiguous()
        torch.testing.assert_close(tp[:, t].reshape(-1, 3), l, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(tv[:, t].reshape(-1, 3), v, rtol=1e-5, atol=1e-6)


def test_run_inference_pos_vel_target_uses_absolute(hip_device, tmp_path):
    ds = dataset(hip_device, tmp_path, double=False, target="pos+vel")
    model = small_model("egnn_mc", hip_device)
    _, locs, vels = I.run_inference("egnn_mc", None, model=model, dataset=ds, save_dir=str(tmp_path / "o"),
                                    device=hip_device, max_rollout_steps=3, print_step=False)
    # frame 1 = the model's absolute prediction from frame 0 (not frame 0 + prediction)
    l0 = torch.tensor(locs[0][:, 0], dtype=torch.float32, device=hip_device).reshape(-1, 3)
    v0 = torch.tensor(vels[0][:, 0], dtype=torch.float32, device=hip_device).reshape(-1, 3)
    out = step_forward(model, "egnn_mc", l0, v0, torch.ones(20, 1, device=hip_device), 4, 5, hip_device)
    np.testing.assert_allclose(locs[1][:, 1].reshape(-1, 3), out[:, :3].double().cpu().numpy(), rtol=1e-5, atol=1e-6)


def test_run_inference_from_checkpoint(hip_device, tmp_path):
    """model=None: load_model_for_inference builds SEGNN() (reference defaults), loads the
    checkpoint's model_state_dict and rolls out in eval mode."""
    torch.manual_seed(3)
    src = SEGNN()
    ckpt = tmp_path / "model.pth"
    torch.save({"model_state_dict": src.state_dict(), "step_count": 1}, ckpt)
    ds = dataset(hip_device, tmp_path, double=False)
    _, locs, vels = I.run_inference("segnn", None, model_path=str(ckpt), dataset=ds, save_dir=str(tmp_path / "o"),
                                    device=hip_device, max_rollout_steps=4, print_step=False)
    m = src.to(hip_device).eval()
    loc0 = torch.tensor(locs[0][:, 0], dtype=torch.float32, device=hip_device)
    vel0 = torch.tensor(vels[0][:, 0], dtype=torch.float32, device=hip_device)
    tp, _ = m.rollout(loc0, vel0, torch.ones(4, 5, 1, device=hip_device), 4)
    np.testing.assert_array_equal(locs[1], tp.cpu().numpy())
    with pytest.raises(ValueError):
        I.run_inference("egnn_mc", None, model_path=str(ckpt), dataset=ds, device=hip_device)
