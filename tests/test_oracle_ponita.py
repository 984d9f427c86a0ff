"""The torch fp64 PONITA oracle (oracle/ponita_torch.py, the gradient reference of the native training
step): pinned to the reference's golden forward, to the numpy oracle, and its autograd gradients to
central finite differences (CPU only)."""
import numpy as np
import pytest
import torch

import nbody_amd.ponita as P
from oracle import ponita as op
from oracle import ponita_torch as opt
from oracle.graph import fc_edge_index


def make(hidden=32, layers=2, **kw):
    torch.manual_seed(0)
    m = P.PONITA_NBODY(hidden_dim=hidden, layers=layers, **kw).double()
    m.model.materialize()
    return m


def ref_params(g, tag):
    pre = tag + "/param/"
    return {k[len(pre):]: g[k] for k in g.files if k.startswith(pre)}


def test_torch_oracle_matches_reference_golden(golden):
    g = golden("ponita")
    p = {k: torch.tensor(np.asarray(v), dtype=torch.float64) for k, v in ref_params(g, "f64").items()}
    pos, vel = torch.tensor(g["loc"]).reshape(-1, 3).double(), torch.tensor(g["vel"]).reshape(-1, 3).double()
    mass = torch.tensor(g["mass"]).reshape(-1, 1).double()
    ei = torch.as_tensor(fc_edge_index(4, 5))
    out = opt.forward(p, mass, vel[:, None], ei, pos[ei[0]] - pos[ei[1]], torch.tensor(g["f64/ori_grid"]), 2)
    np.testing.assert_allclose(out.numpy(), g["f64/pred"], rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("B,N,layers,num_ori,readouts", [(3, 5, 2, 8, True), (2, 4, 3, 6, False)])
def test_torch_oracle_matches_numpy_oracle(B, N, layers, num_ori, readouts):
    m = make(32, layers, num_ori=num_ori, multiple_readouts=readouts)
    params = {k: t.numpy() for k, t in m.state_dict().items()}
    rng = np.random.default_rng(0)
    pos, vel = rng.standard_normal((B * N, 3)), rng.standard_normal((B * N, 3))
    mass = rng.uniform(0.5, 1.5, (B * N, 1))
    ei = fc_edge_index(B, N)
    grid = m.model.ori_grid.numpy()
    ref = op.forward(params, mass, vel[:, None], ei, pos[ei[0]] - pos[ei[1]], grid, layers,
                     multiple_readouts=readouts)
    T = {k: torch.tensor(v) for k, v in params.items()}
    t = torch.tensor
    got = opt.forward(T, t(mass), t(vel)[:, None], t(ei), t(pos[ei[0]] - pos[ei[1]]), t(grid), layers,
                      multiple_readouts=readouts)
    np.testing.assert_allclose(got.numpy(), ref, rtol=1e-12, atol=1e-13)


def test_torch_oracle_gradients_match_finite_differences():
    B, N, layers = 2, 4, 2
    m = make(32, layers, num_ori=6, layer_scale=0.3)
    params = {k: t.numpy().copy() for k, t in m.state_dict().items()}
    rng = np.random.default_rng(3)
    pos, vel = rng.standard_normal((B * N, 3)), rng.standard_normal((B * N, 3))
    mass = rng.uniform(0.5, 1.5, (B * N, 1))
    target = rng.standard_normal((B * N, 6))
    ei = fc_edge_index(B, N)
    grid = m.model.ori_grid.numpy()
    _, _, grads = opt.loss_and_grads(params, grid, pos, vel, mass, ei, target, layers)
    keys = ["model.basis_fn.1.weight", "model.fiber_basis_fn.3.bias", "model.x_embedder.weight",
            "model.interaction_layers.0.conv.kernel.weight", "model.interaction_layers.1.conv.fiber_kernel.weight",
            "model.interaction_layers.0.conv.bias", "model.interaction_layers.1.norm.weight",
            "model.interaction_layers.0.linear_1.bias", "model.interaction_layers.1.linear_2.weight",
            "model.interaction_layers.0.layer_scale", "model.read_out_layers.1.bias"]
    assert set(grads) == {k for k in params if not (k.endswith("callibrated") or k.endswith("ori_grid"))}
    for k in keys:
        flat = params[k].reshape(-1)
        for idx in rng.choice(flat.size, size=min(3, flat.size), replace=False):
            h = 1e-6
            old = flat[idx]
            flat[idx] = old + h
            lp = opt.loss_and_grads(params, grid, pos, vel, mass, ei, target, layers)[0]
            flat[idx] = old - h
            lm = opt.loss_and_grads(params, grid, pos, vel, mass, ei, target, layers)[0]
            flat[idx] = old
            fd = (lp - lm) / (2 * h)
            an = grads[k].reshape(-1)[idx]
            assert abs(fd - an) <= 1e-6 * max(1.0, abs(an)), (k, idx, fd, an)
