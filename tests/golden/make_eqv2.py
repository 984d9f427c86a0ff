"""Generate the EquiformerV2 golden fixtures by running the REFERENCE's own model code.

Run in the build container only (the reference is not on the GPU box):

    python tests/golden/make_eqv2.py [--reference /root/reference]

Imported from the reference (read-only, never copied):
* models/equiformer_v2/architecture/*           (EquiformerV2_nbody and its modules; wigner.py
                                                 reads its Jd.pt with torch.load(weights_only=True))
* utils/build_fully_connected_graph.py
* datasets/nbody/dataset/synthetic_sim.py       (GravitySim, for realistic initial states)

Absent third-party packages are replaced by TEST-ONLY shims:
* e3nn.o3: xyz_to_angles, angles_to_matrix, ToS2Grid, FromS2Grid — oracle/e3nn_so3.py's
  restatement of e3nn's published algorithm (checked here against the reference's own wigner_D).
* torch_geometric.utils.softmax: PyG's segment softmax (src - segment max, exp, / (segment sum +
  1e-16)), restated; torch_geometric.nn.radius_graph / torch_scatter: never called on the path.
The per-edge random gauge of init_edge_rot_mat (edge_rot_mat.py:21, torch.rand_like) is supplied
from a seeded generator and recorded, so the HIP path can be fed the same vectors.

Parameters are overwritten with tests/golden/eqv2_params.param_value so the tests can rebuild
them from the key list alone.  Outputs: tests/golden/eqv2.npz, tests/golden/eqv2_state.json.
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

C4 = dict(num_layers=4, attn_hidden_channels=64, sphere_channels=64, num_heads=4, attn_alpha_channels=8,
          attn_value_channels=4, ffn_hidden_channels=64, lmax_list=[2], mmax_list=[1], grid_resolution=None,
          edge_channels=64, use_atom_edge_embedding=True, share_atom_edge_embedding=False,
          distance_function="projection", num_distance_basis=64, attn_activation="scaled_silu",
          use_s2_act_attn=False, ffn_activation="scaled_silu", max_neighbors=5, max_radius=4096.0, use_pbc=False)
# utils/nbody_utils.py:1324-1361 (load_model_for_inference's EquiformerV2)
INFER = dict(num_layers=3, attn_hidden_channels=32, sphere_channels=32, num_heads=2, attn_alpha_channels=8,
             attn_value_channels=4, ffn_hidden_channels=64, lmax_list=[2], mmax_list=[1], grid_resolution=None,
             edge_channels=32, use_atom_edge_embedding=True, share_atom_edge_embedding=False,
             distance_function="projection", num_distance_basis=64, attn_activation="scaled_silu",
             use_s2_act_attn=False, ffn_activation="scaled_silu", max_neighbors=5, max_radius=4096.0,
             use_pbc=False, alpha_drop=0.01, drop_path_rate=0.0)


def _install_shims(ref):
    import make_golden
    make_golden._install_shims(ref)
    from oracle import e3nn_so3 as E

    def pkg(name, path=None):
        m = sys.modules.get(name) or types.ModuleType(name)
        m.__path__ = [path] if path else []
        sys.modules[name] = m
        return m

    for name in ["models.equiformer_v2", "models.equiformer_v2.architecture"]:
        pkg(name, os.path.join(ref, *name.split(".")))
    e3 = pkg("e3nn")
    o3 = types.ModuleType("e3nn.o3")
    o3.xyz_to_angles, o3.angles_to_matrix = E.xyz_to_angles, E.angles_to_matrix
    o3.ToS2Grid, o3.FromS2Grid = E.ToS2Grid, E.FromS2Grid
    sys.modules["e3nn.o3"] = o3
    e3.o3 = o3

    def softmax(src, index, ptr=None, num_nodes=None, dim=0):
        assert dim == 0
        n = int(index.max()) + 1 if num_nodes is None else num_nodes
        shape = (n,) + tuple(src.shape[1:])
        idx = index.view(-1, *([1] * (src.dim() - 1))).expand_as(src)
        smax = torch.full(shape, float("-inf"), dtype=src.dtype).scatter_reduce(0, idx, src.detach(), "amax",
                                                                              include_self=True)
        out = (src - smax.index_select(0, index)).exp()
        ssum = torch.zeros(shape, dtype=src.dtype).index_add_(0, index, out) + 1e-16
        return out / ssum.index_select(0, index)

    tg = sys.modules["torch_geometric"]
    tg.utils.softmax = softmax
    tg.nn.radius_graph = None
    ts = sys.modules["torch_scatter"]
    ts.segment_coo = ts.segment_csr = None


class Gauge:
    """Replaces torch.rand_like inside init_edge_rot_mat with recorded vectors."""

    def __init__(self, mod):
        self.mod, self.orig = mod, mod.init_edge_rot_mat
        self.queue, self.record = [], []
        mod.init_edge_rot_mat = self

    def __call__(self, vec):
        g = self.queue.pop(0) if self.queue else torch.rand(vec.shape, dtype=torch.float64, generator=self.gen)
        self.record.append(g.clone())
        real = torch.rand_like
        torch.rand_like = lambda t, **kw: g.to(t.dtype)
        try:
            return self.orig(vec)
        finally:
            torch.rand_like = real


def build(mod, cfg, dtype):
    from eqv2_params import param_value
    model = mod.EquiformerV2_nbody(device="cpu", **cfg)
    sd = model.state_dict()
    params = dict(model.named_parameters())
    with torch.no_grad():
        for k, p in params.items():
            p.copy_(torch.from_numpy(param_value(k, p.shape)))
    model = model.to(dtype).eval()
    keys = {k: list(v.shape) for k, v in sd.items()}
    return model, keys, sorted(params)


def initial_states(sim_cls, B, N, seed0):
    sim = sim_cls(n_balls=N, interaction_strength=2, dt=0.01, softening=0.2, noise_var=0)
    tr = [sim.sample_trajectory(T=50, sample_freq=10, random_seed=seed0 + s) for s in range(B)]
    return (np.stack([t[0][0] for t in tr]), np.stack([t[1][0] for t in tr]), np.stack([t[2][0] for t in tr]),
            np.stack([t[3] for t in tr]))


def main():
    sys.dont_write_bytecode = True   # never write __pycache__ into the read-only reference tree
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default=os.environ.get("NBODY_REFERENCE", "/root/reference"))
    a = ap.parse_args()
    _install_shims(a.reference)
    sys.path.insert(0, a.reference)
    mod = importlib.import_module("models.equiformer_v2.architecture.equiformer_v2_nbody")
    so3 = importlib.import_module("models.equiformer_v2.architecture.so3")
    sim_cls = importlib.import_module("datasets.nbody.dataset.synthetic_sim").GravitySim
    gauge = Gauge(mod)
    gauge.gen = torch.Generator().manual_seed(1234)
    out, state = {}, {}

    # ---- Wigner-D of the reference (Jd.pt + angles) for random rotations
    torch.manual_seed(5)
    rot = so3.SO3_Rotation(2)
    vec = torch.randn(16, 3, dtype=torch.float64)
    vec[0] = torch.tensor([0.0, 1.0, 1e-9])           # near the y pole
    R = gauge.orig(vec)
    rot.set_wigner(R)
    out["wigner/rot"], out["wigner/D"] = R.numpy(), rot.wigner.numpy()

    # ---- grid matrices of SO3_Grid(lmax, mmax) as the reference builds them
    for l in range(3):
        for m in range(l + 1):
            g = so3.SO3_Grid(l, m, resolution=None, normalization="component")
            out[f"grid/{l}{m}/to"], out[f"grid/{l}{m}/from"] = g.to_grid_mat.numpy(), g.from_grid_mat.numpy()

    # ---- single forwards
    cases = [("c4", C4, 2, 20, 100), ("inf", INFER, 3, 5, 200)]
    for tag, cfg, B, N, seed in cases:
        loc, vel, force, mass = initial_states(sim_cls, B, N, seed)
        out[f"{tag}/loc"], out[f"{tag}/vel"], out[f"{tag}/mass"] = loc, vel, mass
        for dt, dtype in [("f64", torch.float64), ("f32", torch.float32)]:
            model, keys, pnames = build(mod, cfg, dtype)
            state[tag] = {"config": cfg, "keys": keys, "params": pnames}
            d = [torch.from_numpy(x).to(dtype).reshape(B * N, -1) for x in (loc, vel, force, mass)]
            batch = torch.arange(B).repeat_interleave(N)
            if dt == "f64":
                gauge.queue, gauge.record = [], []
                acts = {}
                hooks = [model.blocks[0].register_forward_hook(lambda m, i, o: acts.__setitem__("block0", o.embedding.clone()))]
                hooks.append(model.edge_degree_embedding.register_forward_hook(
                    lambda m, i, o: acts.__setitem__("edge_degree", o.embedding.clone())))
                hooks.append(model.norm.register_forward_hook(lambda m, i, o: acts.__setitem__("final_norm", o.clone())))
            else:
                gauge.queue, gauge.record = [torch.from_numpy(out[f"{tag}/gauge"])], []
            with torch.no_grad():
                pred = model((d[0], d[1], d[2], d[3], d[0]), batch)
            out[f"{tag}/{dt}/pred"] = pred.numpy()
            if dt == "f64":
                out[f"{tag}/gauge"] = gauge.record[0].numpy()
                for k, v in acts.items():
                    out[f"{tag}/f64/{k}"] = v.numpy()
                for h in hooks:
                    h.remove()

    # ---- self-feed rollout through the tuple branch (infer_self_feed.py:99-194), C4 widths
    B, N, steps = 2, 20, 4
    loc, vel, force, mass = initial_states(sim_cls, B, N, 300)
    model, _, _ = build(mod, C4, torch.float64)
    gauge.queue, gauge.record = [], []
    L, V = [torch.from_numpy(loc)], [torch.from_numpy(vel)]
    F, M = torch.from_numpy(force), torch.from_numpy(mass)
    batch = torch.arange(B).repeat_interleave(N)
    with torch.no_grad():
        for _ in range(steps - 1):
            x = (L[-1].reshape(B * N, 3), V[-1].reshape(B * N, 3), F.reshape(B * N, 3), M.reshape(B * N, 1), None)
            x = (x[0], x[1], x[2], x[3], x[0])
            pred = model(x, batch)
            L.append(L[-1] + pred[:, :3].reshape(B, N, 3))
            V.append(pred[:, 3:].reshape(B, N, 3))
            F = torch.zeros_like(F)
    out["roll/loc0"], out["roll/vel0"], out["roll/force0"], out["roll/mass"] = loc, vel, force, mass
    out["roll/gauge"] = torch.stack(gauge.record).numpy()
    out["roll/loc"], out["roll/vel"] = torch.stack(L, 1).numpy(), torch.stack(V, 1).numpy()

    # ---- the reference's seeded initialisation (torch.manual_seed(0), C4 widths): per parameter the
    # first values and the float64 sum, to pin the RNG consumption order of the module tree
    torch.manual_seed(0)
    ref = mod.EquiformerV2_nbody(device="cpu", **C4)
    names = [k for k, _ in ref.named_parameters()]
    out["seed0/names"] = np.array(names)
    out["seed0/head"] = np.stack([np.pad(p.detach().reshape(-1)[:4].double().numpy(), (0, 4 - min(4, p.numel())))
                                  for _, p in ref.named_parameters()])
    out["seed0/sum"] = np.array([p.detach().double().sum().item() for _, p in ref.named_parameters()])

    np.savez_compressed(os.path.join(HERE, "eqv2.npz"), **out)
    with open(os.path.join(HERE, "eqv2_state.json"), "w") as f:
        json.dump(state, f, indent=1, sort_keys=True)
    print("wrote", len(out), "arrays")


if __name__ == "__main__":
    main()
