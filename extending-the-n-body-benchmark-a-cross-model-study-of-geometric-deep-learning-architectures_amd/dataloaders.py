"""N-body dataloaders of the plugin registry — drop-ins for
dataloaders/{base_dataloader,n_body_dataloader,segnn_n_body_dataloader,
ponita_n_body_dataloader,egnn_mc_n_body_dataloader,equiformer_v2_n_body_dataloader}.py.

``preprocess_batch`` builds the graph the native models consume: positions,
velocities, masses and the (device-built, bit-exact) fully-connected
``edge_index``, plus the family's reference attributes that are pure data
plumbing (PONITA ``x``/``vec``/``rel_pos``, EGNN-MC ``batch``).  Model-specific
featurisation (SEGNN's O3 attributes, EGNN-MC's node/edge features, PONITA's
invariants) happens inside the HIP forward, so it is not materialised here.
``graph.nbx_system_size`` tells the native models the system size without an
edge-index check.
"""
from __future__ import annotations

from abc import ABC, abstractmethod

import torch

from .data import Batch, Data
from .dataset import GravityDatasetOtf
from .graph import build_graph_with_knn

__all__ = ["get_device", "BaseDataLoader", "NBodyDataLoader", "SegnnNBodyDataLoader", "PonitaNBodyDataLoader",
           "EgnnMcNBodyDataLoader", "EquiformerV2NBodyDataLoader"]


def get_device(gpu_id=None):
    """utils/nbody_utils.py:1410-1450 (``'auto'`` picks device 0 here: one process
    per GPU, the launcher sets the visible device)."""
    if isinstance(gpu_id, str):
        if gpu_id.lower() == "auto":
            gpu_id = None
        else:
            try:
                gpu_id = int(gpu_id)
            except ValueError:
                gpu_id = None
    if not torch.cuda.is_available():
        # parameter containers and configs work anywhere; every compute entry point
        # (libnbx) raises on a non-HIP tensor, so nothing silently runs on the CPU
        return torch.device("cpu")
    return torch.device("cuda", 0 if gpu_id is None else int(gpu_id))


class BaseDataLoader(ABC):
    """dataloaders/base_dataloader.py:6-30."""

    def __init__(self, args):
        self.args = args
        self.device = get_device(getattr(args, "gpu_id", None))
        self.dataset = self.create_dataset()
        self.dataset_iter = iter(self.dataset)

    @abstractmethod
    def get_batch(self):
        pass

    @abstractmethod
    def preprocess_batch(self, data, device, training=True):
        pass

    @abstractmethod
    def create_dataset(self):
        pass

    @abstractmethod
    def postprocess_batch(self, predictions, device):
        pass


class NBodyDataLoader(BaseDataLoader):
    """dataloaders/n_body_dataloader.py:9-74."""

    def __init__(self, args, partition="train"):
        super().__init__(args)

    def create_dataset(self):
        a = self.args
        return GravityDatasetOtf(dataset_name=a.dataset_name, num_nodes=a.num_atoms, target=a.target,
                                 sample_freq=a.sample_freq, batch_size=a.batch_size,
                                 double_precision=getattr(a, "precision_mode", "double") == "double",
                                 center_of_mass=a.center_of_mass, use_cached=getattr(a, "model_path", None) is None,
                                 cache_data=True, device=self.device)

    def get_batch(self):
        batch_data = next(self.dataset_iter)
        double = getattr(self.args, "precision_mode", "double") == "double"
        data = [d.view(-1, d.size(2)) for d in batch_data]
        data = [(d.double() if double else d.float()).to(self.device) for d in data]
        loc, vel, force, mass, y = data
        n = self.args.num_atoms
        data_list = [Data(pos=loc[i * n:(i + 1) * n], vel=vel[i * n:(i + 1) * n], force=force[i * n:(i + 1) * n],
                          mass=mass[i * n:(i + 1) * n], y=y[i * n:(i + 1) * n])
                     for i in range(self.args.batch_size)]
        return [Batch.from_data_list(data_list)], None

    def get_num_nodes(self):
        return self.args.num_atoms

    def postprocess_batch(self, predictions, device):
        if isinstance(predictions, torch.Tensor):
            return predictions.to(device)
        return predictions

    def _edges(self, batch, device, num_neighbors):
        n = self.dataset.num_nodes
        batch.edge_index = build_graph_with_knn(batch.pos, self.args.batch_size, n, device, num_neighbors)
        batch.nbx_system_size = n if num_neighbors in (None, n - 1) else None
        return batch


class SegnnNBodyDataLoader(NBodyDataLoader):
    """dataloaders/segnn_n_body_dataloader.py:9-33 (O3Transform runs in the SEGNN kernel)."""

    def preprocess_batch(self, data, device, training=True):
        batch = data.to(device)
        return self._edges(batch, device, self.args.num_neighbors)


class PonitaNBodyDataLoader(NBodyDataLoader):
    """dataloaders/ponita_n_body_dataloader.py:8-38."""

    def preprocess_batch(self, data, device, training=True):
        batch = data.to(device)
        batch.vec = batch.vel.reshape(batch.vel.shape[0], 1, batch.vel.shape[1])
        self._edges(batch, device, self.args.num_neighbors)
        row, col = batch.edge_index
        batch.rel_pos = batch.pos[row] - batch.pos[col]
        batch.x = batch.mass
        return batch


class EgnnMcNBodyDataLoader(NBodyDataLoader):
    """dataloaders/egnn_mc_n_body_dataloader.py:8-61 (node/edge features are built in
    the EGNN-MC kernel; num_neighbors None / <= 0 / >= N means fully connected)."""

    def preprocess_batch(self, data, device, training=True):
        batch = data.to(device)
        n = self.dataset.num_nodes
        k = getattr(self.args, "num_neighbors", None)
        if k is None or k <= 0 or k >= n:
            k = n - 1
        self._edges(batch, device, k)
        if getattr(batch, "batch", None) is None:
            batch.batch = torch.arange(self.args.batch_size, device=device).repeat_interleave(n).long()
        if getattr(batch, "mass", None) is None:
            batch.mass = torch.ones(batch.vel.size(0), 1, device=device, dtype=batch.vel.dtype)
        return batch


class EquiformerV2NBodyDataLoader(NBodyDataLoader):
    """dataloaders/equiformer_v2_n_body_dataloader.py:7-58: kNN (here: min(max_neighbors, N-1))
    edge index, node_type zeros, edge_attr = |pos_row - pos_col|, node_attr = vel, x = mass."""

    def preprocess_batch(self, data, device, training=True):
        batch = data.to(device)
        n_nodes = self.dataset.num_nodes
        k = min(getattr(self.args, "max_neighbors", min(n_nodes - 1, 32)), n_nodes - 1)
        self._edges(batch, device, k)
        row, col = batch.edge_index
        batch.node_type = torch.zeros(self.args.batch_size * n_nodes, dtype=torch.long, device=device)
        batch.edge_attr = torch.norm(batch.pos[row] - batch.pos[col], dim=-1, keepdim=True)
        batch.node_attr = batch.vel
        batch.x = batch.mass
        return batch
