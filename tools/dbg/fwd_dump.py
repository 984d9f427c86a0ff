"""Tuning aid: one C2 SEGNN forward on the GPU, output saved to the given .npy (used to compare
kernel variants selected by environment switches run in separate processes)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import tests.test_gpu_segnn as T  # noqa: E402

dev = torch.device("cuda:0")
model = T.make_model(192, 6, dev, perturb_bn=False)
B, N = int(sys.argv[2]) if len(sys.argv) > 2 else 1024, 5
pos, vel, mass = T.states(B, N, seed=3)
out = T.gpu_forward(model, pos, vel, mass, B, N, dev)
np.save(sys.argv[1], out)
