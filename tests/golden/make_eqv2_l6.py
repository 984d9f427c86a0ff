"""Generate the EquiformerV2 lmax > 2 golden fixtures by running the REFERENCE's own model code.

Run in the build container only (the reference is not on the GPU box):

    python tests/golden/make_eqv2_l6.py [--reference /root/reference]

Same procedure and shims as make_eqv2.py (imported from it), at the reference constructor's default
degrees lmax_list = [6], mmax_list = [2] (equiformer_v2_nbody.py:122-123) and at lmax 4 / mmax 3:
* ``wigner6/rot``, ``wigner6/D``: the reference's SO3_Rotation(6).set_wigner (wigner_D with its Jd.pt)
  for 16 edge frames -- the full 49 x 49 block Wigner matrices;
* ``grid/{l}{m}/to|from`` for l <= 6: SO3_Grid as the reference builds it (its e3nn ToS2Grid /
  FromS2Grid calls go to the oracle/e3nn_so3.py restatement, whose harmonics are pinned to the
  Jd-based D above);
* ``{tag}/...``: single float64 forwards (tuple branch, recorded gauges) of two small models, with
  the block-0 / edge-degree / final-norm activations.
Parameters are overwritten with eqv2_params.param_value.  Outputs: tests/golden/eqv2_l6.npz and
tests/golden/eqv2_l6_state.json.
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

BASE = dict(grid_resolution=None, use_atom_edge_embedding=True, share_atom_edge_embedding=False,
            distance_function="projection", attn_activation="scaled_silu", use_s2_act_attn=False,
            ffn_activation="scaled_silu", max_neighbors=5, max_radius=4096.0, use_pbc=False)
# the reference default degrees (lmax 6, mmax 2) at small widths, and lmax 4 / mmax 3
L6 = dict(BASE, num_layers=2, attn_hidden_channels=32, sphere_channels=32, num_heads=2, attn_alpha_channels=8,
          attn_value_channels=4, ffn_hidden_channels=32, lmax_list=[6], mmax_list=[2], edge_channels=32,
          num_distance_basis=64)
L4 = dict(BASE, num_layers=1, attn_hidden_channels=32, sphere_channels=32, num_heads=4, attn_alpha_channels=8,
          attn_value_channels=4, ffn_hidden_channels=64, lmax_list=[4], mmax_list=[3], edge_channels=32,
          num_distance_basis=64)


def main():
    sys.dont_write_bytecode = True   # never write __pycache__ into the read-only reference tree
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default=os.environ.get("NBODY_REFERENCE", "/root/reference"))
    a = ap.parse_args()
    import make_eqv2 as M
    M._install_shims(a.reference)
    sys.path.insert(0, a.reference)
    mod = importlib.import_module("models.equiformer_v2.architecture.equiformer_v2_nbody")
    so3 = importlib.import_module("models.equiformer_v2.architecture.so3")
    sim_cls = importlib.import_module("datasets.nbody.dataset.synthetic_sim").GravitySim
    gauge = M.Gauge(mod)
    gauge.gen = torch.Generator().manual_seed(4321)
    out, state = {}, {}

    torch.manual_seed(6)
    rot = so3.SO3_Rotation(6)
    vec = torch.randn(16, 3, dtype=torch.float64)
    R = gauge.orig(vec)
    rot.set_wigner(R)
    out["wigner6/rot"], out["wigner6/D"] = R.numpy(), rot.wigner.numpy()

    for l in range(7):
        for m in range(l + 1):
            g = so3.SO3_Grid(l, m, resolution=None, normalization="component")
            out[f"grid/{l}{m}/to"], out[f"grid/{l}{m}/from"] = g.to_grid_mat.numpy(), g.from_grid_mat.numpy()

    for tag, cfg, B, N, seed in [("l6", L6, 2, 5, 500), ("l4", L4, 2, 4, 600)]:
        loc, vel, force, mass = M.initial_states(sim_cls, B, N, seed)
        out[f"{tag}/loc"], out[f"{tag}/vel"], out[f"{tag}/mass"] = loc, vel, mass
        model, keys, pnames = M.build(mod, cfg, torch.float64)
        state[tag] = {"config": cfg, "keys": keys, "params": pnames}
        d = [torch.from_numpy(x).reshape(B * N, -1) for x in (loc, vel, force, mass)]
        batch = torch.arange(B).repeat_interleave(N)
        gauge.queue, gauge.record = [], []
        acts = {}
        hooks = [model.blocks[0].register_forward_hook(lambda m, i, o: acts.__setitem__("block0", o.embedding.clone())),
                 model.edge_degree_embedding.register_forward_hook(
                     lambda m, i, o: acts.__setitem__("edge_degree", o.embedding.clone())),
                 model.norm.register_forward_hook(lambda m, i, o: acts.__setitem__("final_norm", o.clone()))]
        with torch.no_grad():
            pred = model((d[0], d[1], d[2], d[3], d[0]), batch)
        for h in hooks:
            h.remove()
        out[f"{tag}/f64/pred"] = pred.numpy()
        out[f"{tag}/gauge"] = gauge.record[0].numpy()
        for k, v in acts.items():
            out[f"{tag}/f64/{k}"] = v.numpy()
        print(tag, "pred", pred.shape, float(pred.abs().max()))

    np.savez_compressed(os.path.join(HERE, "eqv2_l6.npz"), **out)
    with open(os.path.join(HERE, "eqv2_l6_state.json"), "w") as f:
        json.dump(state, f, indent=1, sort_keys=True)
    print("wrote", len(out), "arrays")


if __name__ == "__main__":
    main()
