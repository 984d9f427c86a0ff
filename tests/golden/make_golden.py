"""Generate golden fixtures by running the REFERENCE's own Python code.

Run in the build container only (the reference is not on the GPU box):

    python tests/golden/make_golden.py [--reference /root/reference]

What is imported from the reference (read-only, never copied):
* utils/build_fully_connected_graph.py          (no shim needed)
* datasets/nbody/dataset/synthetic_sim.py       (GravitySim; utils.nbody_utils is
                                                 stubbed to only provide is_headless,
                                                 because the real module imports
                                                 e3nn-dependent SEGNN)
* models/ponita/**                              (PONITA_NBODY)
* models/egnn_mc/egnn_mc.py                     (EGNNMultiChannel)
* dataloaders/egnn_mc_n_body_dataloader.py      (preprocess_batch)

Absent third-party packages are replaced by the TEST-ONLY shims below:
torch_geometric (Data, MessagePassing.propagate with PyG's source_to_target
semantics: x_j = x[edge_index[0]], x_i = x[edge_index[1]], "add" aggregation at
edge_index[1] along node_dim; Compose; BaseTransform), torch_scatter and
torchmetrics (constructed but never called on the path).  SEGNN needs e3nn and
cannot be imported: no SEGNN fixture comes from the reference.

Outputs: tests/golden/*.npz (small, committed).
"""
from __future__ import annotations

import argparse
import contextlib
import importlib
import inspect
import io
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


# ----------------------------------------------------------------- shims ---
def _install_shims(ref: str):
    def pkg(name, path=None):
        m = types.ModuleType(name)
        m.__path__ = [path] if path else []
        sys.modules[name] = m
        return m

    # namespace-style packages that bypass the reference's eager __init__s
    for name in ["models", "utils", "dataloaders", "datasets", "datasets.nbody", "datasets.nbody.dataset"]:
        pkg(name, os.path.join(ref, *name.split(".")))
    nb = types.ModuleType("utils.nbody_utils")
    nb.is_headless = lambda: True
    sys.modules["utils.nbody_utils"] = nb

    class Data:
        _std = ("x", "edge_index", "edge_attr", "y", "pos", "batch")

        def __init__(self, x=None, **kw):
            if x is not None:
                self.x = x
            for k, v in kw.items():
                setattr(self, k, v)

        def __getattr__(self, k):
            if k in Data._std:
                return None
            raise AttributeError(k)

        def to(self, device, **_):
            for k, v in list(vars(self).items()):
                if torch.is_tensor(v):
                    setattr(self, k, v.to(device))
            return self

    class MessagePassing(torch.nn.Module):
        def __init__(self, aggr="add", node_dim=-2, flow="source_to_target"):
            super().__init__()
            assert aggr == "add" and flow == "source_to_target"
            self.node_dim = node_dim

        def propagate(self, edge_index, **kw):
            src, dst = edge_index[0], edge_index[1]
            margs, n_nodes = {}, None
            for name in inspect.signature(self.message).parameters:
                if name.endswith("_j") or name.endswith("_i"):
                    t = kw[name[:-2]]
                    n_nodes = t.shape[self.node_dim]
                    margs[name] = t.index_select(self.node_dim, src if name.endswith("_j") else dst)
                else:
                    margs[name] = kw[name]
            msg = self.message(**margs)
            shape = list(msg.shape)
            shape[self.node_dim] = n_nodes
            out = msg.new_zeros(shape).index_add_(self.node_dim, dst, msg)
            upd = list(inspect.signature(self.update).parameters)[1:]
            return self.update(out, **{k: kw[k] for k in upd if k in kw})

        def update(self, inputs):
            return inputs

    class Compose:
        def __init__(self, ts):
            self.ts = ts

        def __call__(self, g):
            for t in self.ts:
                g = t(g)
            return g

    class BaseTransform:
        def __call__(self, g):
            return g

    tg = pkg("torch_geometric")
    for sub in ["nn", "data", "transforms", "typing", "utils"]:
        setattr(tg, sub, pkg("torch_geometric." + sub))
    sys.modules["torch_geometric.data"].Data = Data
    sys.modules["torch_geometric.data"].Batch = None
    sys.modules["torch_geometric.nn"].MessagePassing = MessagePassing
    sys.modules["torch_geometric.nn"].global_add_pool = None
    sys.modules["torch_geometric.transforms"].Compose = Compose
    sys.modules["torch_geometric.transforms"].BaseTransform = BaseTransform
    sys.modules["torch_geometric.transforms"].RadiusGraph = None
    sys.modules["torch_geometric.typing"].SparseTensor = None
    for f in ["add_self_loops", "coalesce", "remove_self_loops"]:
        setattr(sys.modules["torch_geometric.utils"], f, None)
    ts = pkg("torch_scatter")
    ts.scatter_mean = ts.scatter = None
    tm = pkg("torchmetrics")
    tm.MeanSquaredError = lambda *a, **k: torch.nn.Identity()
    return Data


def _quiet():
    return contextlib.redirect_stdout(io.StringIO())


# ------------------------------------------------------------- fixtures ---
def make_graph(ref_mods):
    g = ref_mods["graph"]
    out = {}
    for B, N in [(1, 2), (2, 3), (3, 5), (2, 20), (4, 5)]:
        out[f"fc_{B}_{N}"] = g.build_graph_with_knn(torch.zeros(B * N, 3), B, N, "cpu", None).numpy()
    rng = np.random.default_rng(1234)
    for B, N, k in [(2, 6, 3), (3, 8, 2), (1, 5, 1)]:
        loc = rng.standard_normal((B * N, 3))
        out[f"knn_{B}_{N}_{k}_loc"] = loc
        out[f"knn_{B}_{N}_{k}"] = g.build_graph_with_knn(torch.from_numpy(loc), B, N, "cpu", k).numpy()
    try:
        g.build_graph_with_knn(torch.zeros(5, 3), 1, 5, "cpu", 5)
        out["k_ge_n_raises"] = np.array(0)
    except ValueError:
        out["k_ge_n_raises"] = np.array(1)
    np.savez_compressed(os.path.join(HERE, "graph.npz"), **out)


def make_gravity(ref_mods):
    GravitySim = ref_mods["sim"].GravitySim
    out = {}
    for N, T, seeds in [(5, 1000, range(4)), (100, 100, range(2))]:
        sim = GravitySim(n_balls=N, interaction_strength=2, dt=0.01, softening=0.2, noise_var=0)
        for s in seeds:
            p, v, f, m = sim.sample_trajectory(T=T, sample_freq=10, random_seed=s)
            out[f"traj_N{N}_T{T}_s{s}_pos"] = p
            out[f"traj_N{N}_T{T}_s{s}_vel"] = v
            out[f"traj_N{N}_T{T}_s{s}_force"] = f
            out[f"traj_N{N}_T{T}_s{s}_mass"] = m
    rng = np.random.default_rng(7)
    pos = rng.standard_normal((7, 3))
    mass = rng.uniform(0.5, 2.0, (7, 1))
    out["acc_pos"], out["acc_mass"] = pos, mass
    out["acc_out"] = GravitySim.compute_acceleration(pos, mass, 2.0, 0.2)
    np.savez_compressed(os.path.join(HERE, "gravity.npz"), **out)


def make_cache(ref_mods):
    """A ground-truth cache file in the reference's format: the list of B
    ``sample_trajectory`` tuples that GravityDatasetOtf.get_ground_truth_trajectories returns
    (dataset_gravity_otf.py:91-107), written with the reference's own call
    ``pickle.dump(data, file)`` (_save_simulations, :118-135) into
    ``<data_path>/<sha256 of the constructor arguments>/0.pkl`` (:52-56,176-183).  The
    reference module itself cannot be imported here (matplotlib is absent and importing it
    creates a directory inside the read-only reference tree), so the folder name is computed
    by the same json/sha256 rule and the trajectories come from the reference's GravitySim."""
    import hashlib
    import json
    import pickle
    GravitySim = ref_mods["sim"].GravitySim
    kw = {"dataset_name": "nbody_small", "target": "pos_dt+vel", "batch_size": 3, "sim_length": 200,
          "sample_freq": 10, "noise_var": 0, "num_nodes": 5, "vel_norm": 1e-16, "interaction_strength": 2,
          "dt": 0.01, "softening": 0.2, "double_precision": False, "center_of_mass": False, "lmax_attr": 1}
    folder = hashlib.sha256(json.dumps(kw, sort_keys=True).encode()).hexdigest()
    sim = GravitySim(noise_var=0, n_balls=5, vel_norm=1e-16, interaction_strength=2, dt=0.01, softening=0.2)
    data = [sim.sample_trajectory(200, 10, random_seed=s) for s in (11, 12, 13)]
    d = os.path.join(HERE, "ref_cache", folder)
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "0.pkl"), "wb") as f:
        pickle.dump(data, f)


def _initial_states(sim_cls, B, N, T=100):
    sim = sim_cls(n_balls=N, interaction_strength=2, dt=0.01, softening=0.2, noise_var=0)
    trajs = [sim.sample_trajectory(T=T, sample_freq=10, random_seed=s) for s in range(B)]
    loc = np.stack([t[0][0] for t in trajs])
    vel = np.stack([t[1][0] for t in trajs])
    force = np.stack([t[2][0] for t in trajs])
    mass = np.stack([t[3] for t in trajs])
    return loc, vel, force, mass


def _rollout(step, loc0, vel0, force0, mass0, steps, dtype):
    """Mirror of infer_self_feed.py:99-194 (target pos_dt+vel)."""
    B, N, D = loc0.shape
    locs, vels = [torch.from_numpy(loc0).to(dtype)], [torch.from_numpy(vel0).to(dtype)]
    force, mass = torch.from_numpy(force0).to(dtype), torch.from_numpy(mass0).to(dtype)
    for _ in range(steps - 1):
        pred = step(locs[-1].reshape(B * N, D), vels[-1].reshape(B * N, D), force.reshape(B * N, D),
                    mass.reshape(B * N, 1), B, N)
        locs.append(locs[-1] + pred[..., :3].reshape(B, N, D))
        vels.append(pred[..., 3:].reshape(B, N, D))
        force = torch.zeros_like(locs[-1])
    return torch.stack(locs, 1).numpy(), torch.stack(vels, 1).numpy()


def make_ponita(ref_mods, Data):
    PONITA_NBODY = ref_mods["ponita"].PONITA_NBODY
    g = ref_mods["graph"]
    loc, vel, force, mass = _initial_states(ref_mods["sim"].GravitySim, 4, 5)
    out = {"loc": loc, "vel": vel, "force": force, "mass": mass}
    for tag, dtype in [("f64", torch.float64), ("f32", torch.float32)]:
        torch.manual_seed(0)
        with _quiet():
            model = PONITA_NBODY(hidden_dim=32, layers=2, lr=1e-3)
        model = model.to(dtype)

        def step(l, v, f, m, B, N):
            graph = Data(torch.hstack([m]))
            graph.pos = l
            graph.vec = v.reshape(v.shape[0], 1, v.shape[1])
            ei = g.build_graph_with_knn(l, B, N, "cpu", N - 1)
            graph.edge_index = ei
            graph.rel_pos = l[ei[0]] - l[ei[1]]
            return model(graph)

        B, N = loc.shape[:2]
        l0 = torch.from_numpy(loc).to(dtype).reshape(-1, 3)
        v0 = torch.from_numpy(vel).to(dtype).reshape(-1, 3)
        m0 = torch.from_numpy(mass).to(dtype).reshape(-1, 1)
        with torch.no_grad(), _quiet():
            step(l0, v0, None, m0, B, N)          # materialise LazyLinear + one-time "callibrate"
            pred = step(l0, v0, None, m0, B, N)
            L, Vv = _rollout(step, loc, vel, force, mass, 10, dtype)
        for k, t in model.state_dict().items():
            out[f"{tag}/param/{k}"] = t.numpy()
        out[f"{tag}/ori_grid"] = model.model.transform.ts[0].ori_grid_s2.to(dtype).numpy()
        out[f"{tag}/pred"] = pred.numpy()
        out[f"{tag}/roll_loc"], out[f"{tag}/roll_vel"] = L, Vv
    np.savez_compressed(os.path.join(HERE, "ponita.npz"), **out)


def make_egnn_mc(ref_mods, Data):
    EGNN = ref_mods["egnn"].EGNNMultiChannel
    DL = ref_mods["egnn_dl"].EgnnMcNBodyDataLoader
    g = ref_mods["graph"]
    loc, vel, force, mass = _initial_states(ref_mods["sim"].GravitySim, 4, 5)
    out = {"loc": loc, "vel": vel, "force": force, "mass": mass}
    for tag, dtype in [("f64", torch.float64), ("f32", torch.float32)]:
        torch.manual_seed(0)
        model = EGNN(node_input_dim=2, edge_attr_dim=4, hidden_node_dim=32, hidden_edge_dim=32,
                     hidden_coord_dim=32, num_layers=2, target_names=("pos_dt", "vel"),
                     activation="silu", coords_weight=1.0, recurrent=True, norm_diff=True, tanh=True,
                     device="cpu").to(dtype)
        fake = types.SimpleNamespace(args=types.SimpleNamespace(batch_size=loc.shape[0], num_neighbors=None),
                                     dataset=types.SimpleNamespace(num_nodes=loc.shape[1]))

        def step(l, v, f, m, B, N):
            graph = Data(pos=l, vel=v, force=f, mass=m)
            graph.batch = torch.arange(B).repeat_interleave(N).long()
            graph = DL.preprocess_batch(fake, graph, device="cpu", training=False)
            return model(graph)

        B, N = loc.shape[:2]
        with torch.no_grad():
            pred = step(torch.from_numpy(loc).to(dtype).reshape(-1, 3), torch.from_numpy(vel).to(dtype).reshape(-1, 3),
                        torch.from_numpy(force).to(dtype).reshape(-1, 3), torch.from_numpy(mass).to(dtype).reshape(-1, 1), B, N)
            L, Vv = _rollout(step, loc, vel, force, mass, 10, dtype)
        for k, t in model.state_dict().items():
            out[f"{tag}/param/{k}"] = t.numpy()
        out[f"{tag}/pred"] = pred.numpy()
        out[f"{tag}/roll_loc"], out[f"{tag}/roll_vel"] = L, Vv
    np.savez_compressed(os.path.join(HERE, "egnn_mc.npz"), **out)


def make_egnn_grad(ref_mods, Data):
    """Parameter gradients of the reference EGNNMultiChannel (float64 autograd) for
    loss = sum(pred * G) with a seeded G, i.e. dL/dpred = G: the fixture of the native
    training backward (csrc/egnn_train.hip).  Two widths; N = 5 and 6."""
    EGNN = ref_mods["egnn"].EGNNMultiChannel
    DL = ref_mods["egnn_dl"].EgnnMcNBodyDataLoader
    out = {}
    for tag, (H, L, B, N) in {"h32": (32, 2, 4, 5), "h64": (64, 3, 3, 6)}.items():
        loc, vel, force, mass = _initial_states(ref_mods["sim"].GravitySim, B, N)
        torch.manual_seed(1)
        model = EGNN(node_input_dim=2, edge_attr_dim=4, hidden_node_dim=H, hidden_edge_dim=H, hidden_coord_dim=H,
                     num_layers=L, target_names=("pos_dt", "vel"), activation="silu", coords_weight=1.0,
                     recurrent=True, norm_diff=True, tanh=True, device="cpu").double()
        fake = types.SimpleNamespace(args=types.SimpleNamespace(batch_size=B, num_neighbors=None),
                                     dataset=types.SimpleNamespace(num_nodes=N))
        graph = Data(pos=torch.from_numpy(loc).reshape(-1, 3), vel=torch.from_numpy(vel).reshape(-1, 3),
                     force=torch.from_numpy(force).reshape(-1, 3), mass=torch.from_numpy(mass).reshape(-1, 1))
        graph.batch = torch.arange(B).repeat_interleave(N).long()
        graph = DL.preprocess_batch(fake, graph, device="cpu", training=True)
        pred = model(graph)
        G = torch.from_numpy(np.random.default_rng(5).standard_normal(pred.shape))
        (pred * G).sum().backward()
        out[f"{tag}/loc"], out[f"{tag}/vel"], out[f"{tag}/mass"] = loc, vel, mass
        out[f"{tag}/G"], out[f"{tag}/pred"] = G.numpy(), pred.detach().numpy()
        for k, prm in model.named_parameters():
            out[f"{tag}/param/{k}"] = prm.detach().numpy()
            out[f"{tag}/grad/{k}"] = prm.grad.numpy()
    np.savez_compressed(os.path.join(HERE, "egnn_mc_grad.npz"), **out)


def main():
    sys.dont_write_bytecode = True   # never write __pycache__ into the read-only reference tree
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default=os.environ.get("NBODY_REFERENCE", "/root/reference"))
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    Data = _install_shims(a.reference)
    sys.path.insert(0, a.reference)
    mods = {
        "graph": importlib.import_module("utils.build_fully_connected_graph"),
        "sim": importlib.import_module("datasets.nbody.dataset.synthetic_sim"),
    }
    jobs = {"graph": make_graph, "gravity": make_gravity, "cache": make_cache}
    if a.only in (None, "ponita"):
        mods["ponita"] = importlib.import_module("models.ponita.ponita_nbody")
    if a.only in (None, "egnn_mc"):
        mods["egnn"] = importlib.import_module("models.egnn_mc.egnn_mc")
        mods["egnn_dl"] = importlib.import_module("dataloaders.egnn_mc_n_body_dataloader")
    for name, fn in jobs.items():
        if a.only in (None, name):
            fn(mods)
    if a.only in (None, "ponita"):
        make_ponita(mods, Data)
    if a.only in (None, "egnn_mc"):
        make_egnn_mc(mods, Data)
    if a.only in ("egnn_grad",):
        mods["egnn"] = importlib.import_module("models.egnn_mc.egnn_mc")
        mods["egnn_dl"] = importlib.import_module("dataloaders.egnn_mc_n_body_dataloader")
        make_egnn_grad(mods, Data)


if __name__ == "__main__":
    main()
