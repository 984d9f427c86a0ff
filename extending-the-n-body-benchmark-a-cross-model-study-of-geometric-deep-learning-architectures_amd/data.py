"""Minimal graph container with the torch_geometric ``Data`` / ``Batch`` surface the
N-body dataloaders and the rollout use (attribute bag, ``.to(device)``,
``Batch.from_data_list`` concatenating node tensors and building ``batch``).
torch_geometric is not a dependency of this package."""
from __future__ import annotations

import torch

__all__ = ["Data", "Batch"]


class Data:
    def __init__(self, x=None, **kwargs):
        if x is not None:
            self.x = x
        for k, v in kwargs.items():
            setattr(self, k, v)

    def keys(self):
        return [k for k in vars(self) if not k.startswith("_")]

    def to(self, device):
        for k in self.keys():
            v = getattr(self, k)
            if isinstance(v, torch.Tensor):
                setattr(self, k, v.to(device))
        return self

    @property
    def num_nodes(self):
        for k in ("pos", "x", "vel"):
            v = getattr(self, k, None)
            if isinstance(v, torch.Tensor):
                return v.shape[0]
        return None

    def __repr__(self):
        parts = []
        for k in self.keys():
            v = getattr(self, k)
            parts.append(f"{k}={list(v.shape)}" if isinstance(v, torch.Tensor) else f"{k}={v!r}")
        return f"{type(self).__name__}({', '.join(parts)})"


class Batch(Data):
    @classmethod
    def from_data_list(cls, data_list):
        out = cls()
        keys = data_list[0].keys()
        for k in keys:
            vals = [getattr(d, k) for d in data_list]
            if all(isinstance(v, torch.Tensor) for v in vals):
                setattr(out, k, torch.cat(vals, 0))
        sizes = [d.num_nodes for d in data_list]
        device = getattr(out, keys[0]).device if keys else None
        out.batch = torch.repeat_interleave(torch.arange(len(sizes), device=device),
                                            torch.tensor(sizes, device=device))
        out.num_graphs = len(data_list)
        return out
