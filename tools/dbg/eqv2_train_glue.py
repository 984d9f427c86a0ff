"""Count the torch (non-libnbx) kernels one eager EquiformerV2 C4 training step launches, grouped by
the Python line that issued them (torch.profiler).  Diagnostic for the launch-bound training step."""
import collections
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from nbody_amd.equiformer_v2 import EquiformerV2_nbody  # noqa: E402
import nbody_amd.eqv2_train as ET  # noqa: E402

dev = torch.device("cuda:0")
B, N = 64, 5
torch.manual_seed(0)
model = EquiformerV2_nbody(**bench.EQV2_C4).to(dev).train()
loc, vel, mass = bench.initial_states(B, N, 0)
t = lambda x: torch.tensor(x, dtype=torch.float32, device=dev)
pos, vv, q = t(loc.reshape(-1, 3)), t(vel.reshape(-1, 3)), t(mass.reshape(-1))
gauge = t(np.random.default_rng(0).uniform(0, 1, (B * N * (N - 1), 3)))
target = t(np.random.default_rng(1).standard_normal((B * N, 6)) * 0.1)


def step():
    model.zero_grad(set_to_none=True)
    loss = torch.nn.functional.mse_loss(ET.train_forward(model, pos, vv, q, B, N, gauge, 0), target)
    loss.backward()


step()
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402
with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
    step()
    torch.cuda.synchronize()
cnt = collections.Counter()
for ev in prof.events():
    if not ev.name.startswith("aten::") or ev.name in ("aten::empty", "aten::empty_strided", "aten::view",
                                                        "aten::as_strided", "aten::_reshape_alias", "aten::reshape",
                                                        "aten::select", "aten::slice", "aten::detach", "aten::t",
                                                        "aten::transpose", "aten::expand", "aten::unsqueeze",
                                                        "aten::squeeze", "aten::permute", "aten::alias", "aten::lift_fresh",
                                                        "aten::is_nonzero", "aten::item", "aten::_local_scalar_dense",
                                                        "aten::resolve_conj", "aten::resolve_neg"):
        continue
    if ev.cpu_parent is not None and ev.cpu_parent.name.startswith("aten::"):
        continue   # count top-level aten ops only
    frame = next((f for f in (ev.stack or []) if "nbody_amd" in f or "eqv2" in f or "segnn_train" in f
                  or "ponita_train" in f), "?")
    cnt[(ev.name, frame.split("/")[-1][:90])] += 1
total = sum(cnt.values())
print("top-level aten ops in one step:", total)
for (name, frame), c in cnt.most_common(45):
    print(f"{c:5d}  {name:32s} {frame}")
