"""Per-column fp32 error envelope of the small SEGNN forward configurations (build container, CPU only).

    python tests/golden/make_segnn_small_ensemble.py

tests/test_gpu_segnn.py::test_forward_matches_oracle checks each small configuration (20-160 nodes, up
to 3 layers, train-mode BatchNorm over those few nodes) per output column against the fp64 oracle.  How
far an fp32 computation of those forwards can land from fp64 is measured here, not assumed: for every
configuration the torch restatement oracle/segnn_torch.py runs in fp32 as several equally valid fp32
computations of the same forward -- natural order, systems permuted, edge list shuffled, and the
contraction axis of every tensor-product GEMM permuted -- and the worst per-column error / column scale
(the metric of assert_close_cols) of each is stored.  The models and inputs are the test's own
(make_model(hidden, layers, perturb_bn=True, seed 0), states(B, N, seed 0)).  The oracle is the e3nn
restatement: parity vs e3nn itself is UNPINNED (e3nn is absent from this image).

Output: tests/golden/segnn_small_ensemble.json  {config key: {"members": {name: worst rel}, "max": .., "median": ..}}
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "tests"))

CONFIGS = [(16, 1, 2, 5, True), (32, 2, 4, 5, True), (64, 3, 8, 5, False), (192, 6, 16, 5, True),
           (192, 6, 3, 2, True), (24, 2, 3, 7, True), (192, 2, 2, 20, True)]


def key(c):
    return "h{}_l{}_b{}_n{}_{}".format(c[0], c[1], c[2], c[3], "train" if c[4] else "eval")


def worst_col(got, ref):
    err = np.abs(got - ref).max(0)
    scale = np.maximum(np.abs(ref).max(0), 1e-30)
    return float((err / scale).max())


def main():
    import oracle.segnn_torch as ST
    from make_segnn_c2_ensemble import _fctp_kperm
    from oracle.graph import fc_edge_index
    from oracle.segnn import SEGNNOracle, o3_transform
    torch.set_num_threads(8)
    out = {}
    for hidden, layers, B, N, training in CONFIGS:
        torch.manual_seed(0)
        import nbody_amd.segnn as S
        from test_gpu_segnn import make_model, params_of, states
        model = make_model(hidden, layers, torch.device("cpu"))
        params = params_of(model)
        pos, vel, mass = states(B, N)
        om = SEGNNOracle(hidden_features=hidden, num_layers=layers)
        ei0 = fc_edge_index(B, N)
        x, ea, na, amf = o3_transform(pos, vel, mass, ei0)
        ref, _ = om.forward(params, x, ei0, ea, na, amf, training=training)
        members = {}
        for kind, n in (("plain", 1), ("sysperm", 3), ("edgeperm", 3), ("kperm", 4)):
            for i in range(n):
                rng = np.random.default_rng(1000 * len(members) + i)
                perm = rng.permutation(B) if kind == "sysperm" else np.arange(B)
                idx = (perm[:, None] * N + np.arange(N)).reshape(-1)
                inv = np.argsort(idx)
                ei = fc_edge_index(B, N)
                if kind == "edgeperm":
                    ei = ei[:, rng.permutation(ei.shape[1])]
                P = {k: torch.tensor(v, dtype=torch.float32) for k, v in params.items()}
                saved = ST.fctp
                if kind == "kperm":
                    ST.fctp = _fctp_kperm(rng)
                try:
                    with torch.no_grad():
                        t = lambda a: torch.tensor(a[idx], dtype=torch.float32)
                        o, _ = ST.forward(om, P, t(pos), t(vel), t(mass), torch.as_tensor(ei), training)
                finally:
                    ST.fctp = saved
                members[f"{kind}-{i}"] = worst_col(o.double().numpy()[inv], ref)
        vals = np.array(list(members.values()))
        out[key((hidden, layers, B, N, training))] = {"members": members, "max": float(vals.max()),
                                                     "median": float(np.median(vals))}
        print(key((hidden, layers, B, N, training)), f"max {vals.max():.2e} median {np.median(vals):.2e}",
              flush=True)
    with open(os.path.join(HERE, "segnn_small_ensemble.json"), "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
