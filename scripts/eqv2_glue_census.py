"""Diagnosis: census of the torch (non-library) ops one EquiformerV2 training step (bench.py
--model eqv2_train, B = 64) dispatches: each aten op with its forward source line in eqv2_train.py
or the autograd node that ran it in the backward, counted per step."""
import collections
import os
import sys
import traceback

import numpy as np
import torch
from torch.utils._python_dispatch import TorchDispatchMode

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

SKIP = {"aten.view", "aten._unsafe_view", "aten.t", "aten.transpose", "aten.detach", "aten.split_with_sizes",
        "aten.split", "aten.unbind", "aten.slice", "aten.select", "aten.as_strided", "aten.expand",
        "aten.unsqueeze", "aten.squeeze", "aten.permute", "aten.alias", "aten.empty", "aten.empty_strided",
        "aten.empty_like", "aten.new_empty", "aten.new_empty_strided", "aten.reshape", "aten._to_copy?",
        "aten.narrow", "aten.lift_fresh", "aten.is_same_size", "aten._has_compatible_shallow_copy_type"}


class Census(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.c = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func.overloadpacket).replace("aten::", "aten.")
        out = func(*args, **(kwargs or {}))
        if name in SKIP:
            return out
        node = torch._C._current_autograd_node()
        if node is not None:
            where = "bw:" + type(node).__name__
        else:
            fr = [f for f in traceback.extract_stack()[:-1] if "eqv2_train.py" in f.filename or "bench.py" in f.filename]
            where = f"fw:{os.path.basename(fr[-1].filename)}:{fr[-1].lineno}" if fr else "fw:?"
        self.c[(name, where)] += 1
        return out


def main():
    from nbody_amd.equiformer_v2 import EquiformerV2_nbody
    import nbody_amd.eqv2_train as ET
    dev = torch.device("cuda:0")
    B, N = 64, 5
    torch.manual_seed(0)
    model = EquiformerV2_nbody(**bench.EQV2_C4).to(dev).train()
    loc, vel, mass = bench.initial_states(B, N, 0)
    rng = np.random.default_rng(300)
    t = lambda x: torch.tensor(x, dtype=torch.float32, device=dev)
    pos, vv, q = t(loc.reshape(-1, 3)), t(vel.reshape(-1, 3)), t(mass.reshape(-1, 1))
    gauge = t(rng.uniform(0, 1, (B * N * (N - 1), 3)))
    target = t(rng.standard_normal((B * N, 6)) * 0.1)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, fused=True)
    params = list(model.parameters())

    def step():
        opt.zero_grad(set_to_none=True)
        loss = torch.nn.functional.mse_loss(ET.train_forward(model, pos, vv, q.reshape(-1), B, N, gauge, 0), target)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(params, 1.0, foreach=True)
        opt.step()

    step()
    torch.cuda.synchronize()
    cen = Census()
    with cen:
        step()
    torch.cuda.synchronize()
    tot = sum(cen.c.values())
    byop = collections.Counter()
    for (n, _), k in cen.c.items():
        byop[n] += k
    print(f"torch ops per step (views excluded): {tot}")
    for n, k in byop.most_common(40):
        print(f"  {k:5d} {n}")
    print("by site:")
    for (n, w), k in cen.c.most_common(120):
        print(f"  {k:5d} {n:32s} {w}")


if __name__ == "__main__":
    main()
