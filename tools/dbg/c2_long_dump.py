"""Dump the device C2 long-horizon rollout (tests/golden/segnn_c2_long.npz workload) for offline
analysis of the error measures: gpurun_out/c2_long_device.npz (slice trajectories, fp32)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import nbody_amd.segnn as S  # noqa: E402

fx = np.load(os.path.join(ROOT, "tests", "golden", "segnn_c2_long.npz"))
dev = torch.device("cuda:0")
torch.manual_seed(0)
model = S.SEGNN(hidden_features=192, num_layers=6, deterministic=True)
with torch.no_grad():
    model.pre_pool2.tp.weight.mul_(float(fx["scale"]))
model = model.to(dev).train()
S_, T = fx["traj_loc"].shape[:2]
t = lambda a: torch.tensor(a, dtype=torch.float32, device=dev)
loc0 = fx["loc0"]
tp, tv = model.rollout(t(loc0), t(fx["vel0"]), t(np.ones(loc0.shape[:2] + (1,))), T)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "c2_long_device.npz"), tp=tp[:S_].cpu().numpy(),
                    tv=tv[:S_].cpu().numpy())
print("saved", tp.shape)
