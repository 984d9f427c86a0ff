"""Per-wave phase clocks of the SEGNN C2 kernels (NBX_TP_DEBUG=1: each tensor-product launch prints its
average staging / K-loop / epilogue clocks and the waves' span to stderr).  Runs two train-mode C2
forwards (B = 1024) and keeps the second's lines.
usage: NBX_TP_DEBUG=1 python scripts/tp_phase_clocks.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

if __name__ == "__main__":
    assert os.environ.get("NBX_TP_DEBUG"), "set NBX_TP_DEBUG=1"
    import torch
    import test_gpu_segnn as T
    dev = torch.device("cuda:0")
    model = T.make_model(192, 6, dev, perturb_bn=False).train()
    pos, vel, mass = T.states(1024, 5, seed=3)
    for i in range(2):
        print(f"---- forward {i}", file=sys.stderr, flush=True)
        out = T.gpu_forward(model, pos, vel, mass, 1024, 5, dev)
    assert np.isfinite(out).all()
