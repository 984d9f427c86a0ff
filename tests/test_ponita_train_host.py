"""CPU check of the PONITA training composition (ponita_train.py, host logic): with every native
operator swapped for its torch definition (fp64), ``train_forward`` equals the torch fp64 oracle
(oracle/ponita_torch.py) and its autograd gradients equal the oracle's.  The native operators
themselves are checked on the GPU (tests/test_gpu_ponita_train.py)."""
import numpy as np
import pytest
import torch

import nbody_amd.ponita as P
import nbody_amd.ponita_train as T
from oracle import ponita_torch as OT
from oracle.graph import fc_edge_index, knn_edge_index


class _G:
    def __init__(self, ei, V, device=None):
        ei = torch.as_tensor(ei)
        self.src, self.dst, self.V, self.E = ei[0].long(), ei[1].long(), V, ei.shape[1]


def _fn(f):
    return type("F", (), {"apply": staticmethod(f)})


def _linear(X, W, b=None, act=0, ldx=None):
    K = W.shape[1]
    y = X[:, :K] @ W.T
    if b is not None:
        y = y + b
    return OT.gelu(y) if act == 1 else y


def _featurize(pos, vel, mass, ori, g):
    attr, fib = OT.invariants(ori, pos[g.src] - pos[g.dst])
    pa = OT.poly_features(attr).reshape(-1, 14)
    pf = OT.poly_features(fib).reshape(-1, 3)
    O = ori.shape[0]
    lift = torch.stack([mass.repeat_interleave(O), (vel @ ori.T).reshape(-1)], 1)
    return pa, pf, lift


def _message(K, H, g, O):
    C = H.shape[1]
    return torch.zeros(g.V, O, C, dtype=H.dtype).index_add(
        0, g.dst, K.view(g.E, O, C) * H.view(g.V, O, C)[g.src]).reshape(-1, C)


def _fiber(X1, FK, bias, O):
    C = X1.shape[1]
    return (torch.einsum("boc,opc->bpc", X1.view(-1, O, C), FK.view(O, O, C)) / O + bias).reshape(-1, C)


@pytest.fixture
def torch_ops(monkeypatch):
    monkeypatch.setattr(T, "_f32", torch.float64)
    monkeypatch.setattr(T, "Graph", _G)
    monkeypatch.setattr(T, "featurize", _featurize)
    monkeypatch.setattr(T, "linear", _linear)
    monkeypatch.setattr(T, "_MessageFn", _fn(_message))
    monkeypatch.setattr(T, "_FiberFn", _fn(_fiber))
    monkeypatch.setattr(T, "_LayerNormFn", _fn(lambda X, w, b, eps: OT.layer_norm(X, w, b, eps)))


@pytest.mark.parametrize("knn", [False, True])
def test_train_forward_composition_matches_oracle(torch_ops, knn):
    torch.manual_seed(0)
    m = P.PONITA_NBODY(hidden_dim=32, layers=2, num_ori=6, layer_scale=0.3).double()
    m.model.materialize()
    B, N = 3, 5
    rng = np.random.default_rng(1)
    pos = torch.tensor(rng.standard_normal((B * N, 3)))
    vel = torch.tensor(rng.standard_normal((B * N, 3)))
    mass = torch.tensor(rng.uniform(0.5, 1.5, B * N))
    ei = knn_edge_index(pos.numpy(), B, N, 2) if knn else fc_edge_index(B, N)
    ei = torch.as_tensor(ei)
    got = T.train_forward(m, pos, vel, mass, ei)
    (got ** 2).sum().backward()
    grads = {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}
    Pm = {k: v.detach().clone().requires_grad_(not (k.endswith("callibrated") or k.endswith("ori_grid")))
          for k, v in m.state_dict().items()}
    ref = OT.forward(Pm, mass[:, None], vel[:, None], ei, pos[ei[0]] - pos[ei[1]], Pm["model.ori_grid"], 2)
    (ref ** 2).sum().backward()
    torch.testing.assert_close(got.detach(), ref.detach(), rtol=0, atol=1e-13)
    rg = {k: v.grad for k, v in Pm.items() if v.grad is not None}
    assert set(grads) == set(rg)
    for k in rg:
        torch.testing.assert_close(grads[k], rg[k], rtol=1e-10, atol=1e-12, msg=k)
