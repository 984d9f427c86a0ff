"""Quick per-model rollout timing on one GPU (development aid, not the bench contract)."""
import argparse
import json
import sys
import time

import torch

sys.path.insert(0, ".")
import nbody_amd  # noqa: F401
from nbody_amd.ponita import PONITA_NBODY
from nbody_amd.egnn_mc import EGNNMultiChannel


def run(name, model, B, N, frames, dev):
    torch.manual_seed(1)
    loc = torch.randn(B, N, 3, device=dev)
    vel = torch.randn(B, N, 3, device=dev) * 0.1
    mass = torch.ones(B, N, 1, device=dev)
    model.rollout(loc, vel, mass, 3)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    model.rollout(loc, vel, mass, frames + 1)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"model": name, "B": B, "N": N, "steps": frames, "ms_per_step": 1e3 * dt / frames,
                      "steps_per_s": frames / dt}), flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--ponita_B", type=int, default=4096)
    ap.add_argument("--only", default="ponita,egnn")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    if "ponita" in a.only:
        torch.manual_seed(0)
        m = PONITA_NBODY(hidden_dim=128, layers=6).to(dev)
        m.eval()
        run("ponita_C3", m, a.ponita_B, 5, a.frames, dev)
    if "egnn" not in a.only:
        raise SystemExit(0)
    torch.manual_seed(0)
    e = EGNNMultiChannel(node_input_dim=2, edge_attr_dim=4, hidden_node_dim=128, hidden_edge_dim=128,
                         hidden_coord_dim=128, num_layers=6, target_names=("pos_dt", "vel"), norm_diff=True,
                         tanh=True).to(dev)
    run("egnn_mc_C1", e, 64, 5, 100, dev)
    run("egnn_mc_B1024", e, 1024, 5, 100, dev)
