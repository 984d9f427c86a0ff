"""Drop-in for utils/build_fully_connected_graph.py, edge indices built on the device
by libnbx (bit-exact with the reference)."""
from __future__ import annotations

from collections import OrderedDict

import torch

from . import _lib

_CACHE_MAX = 8
_cache: "OrderedDict[tuple, torch.Tensor]" = OrderedDict()


def _fc_edge_index_shared(batch_size: int, num_nodes: int, device) -> torch.Tensor:
    """Internal read-only copy of the fully-connected pattern, cached per (B, N, device)
    (LRU, at most _CACHE_MAX entries).  Used by the models to validate a graph's
    edge_index; never handed to callers."""
    device = torch.device(device)
    key = (int(batch_size), int(num_nodes), device)
    ei = _cache.get(key)
    if ei is None:
        E = batch_size * num_nodes * (num_nodes - 1)
        ei = torch.empty(2, E, dtype=torch.int64, device=device)
        _lib.check(_lib.lib().nbx_fc_edge_index(batch_size, num_nodes, _lib.dev_ptr(ei), _lib.stream_ptr(device)),
                   "nbx_fc_edge_index")
        _cache[key] = ei
        while len(_cache) > _CACHE_MAX:
            _cache.popitem(last=False)
    else:
        _cache.move_to_end(key)
    return ei


def fc_edge_index(batch_size: int, num_nodes: int, device) -> torch.Tensor:
    """_build_fully_connected_edge_index (build_fully_connected_graph.py:4-20).
    Returns a fresh tensor on every call, like the reference (callers may modify it
    in place, e.g. to offset indices while collating)."""
    return _fc_edge_index_shared(batch_size, num_nodes, device).clone()


def build_graph_with_knn(loc, batch_size, num_nodes, device, num_neighbors):
    """build_graph_with_knn (build_fully_connected_graph.py:23-80)."""
    num_nodes = int(num_nodes)
    k = num_nodes - 1 if num_neighbors is None else int(num_neighbors)
    if k >= num_nodes:
        raise ValueError("Graph cannot have more neighbors than there are nodes in simulation - 1")
    if k == num_nodes - 1:
        return fc_edge_index(batch_size, num_nodes, device)
    loc = loc.reshape(batch_size * num_nodes, -1).contiguous()
    if loc.dtype not in (torch.float32, torch.float64):
        raise TypeError("loc must be fp32 or fp64")
    ei = torch.empty(2, batch_size * num_nodes * k, dtype=torch.int64, device=loc.device)
    _lib.check(_lib.lib().nbx_knn_edge_index(_lib.dev_ptr(loc), 0 if loc.dtype == torch.float32 else 1,
                                             batch_size, num_nodes, k, _lib.dev_ptr(ei), _lib.stream_ptr(loc.device)),
               "nbx_knn_edge_index")
    return ei.to(device)


def system_layout(graph, num_nodes: int, num_edges: int, device):
    """(B, N, fully_connected) of a batched graph of equal-size systems, for the native models.
    N comes from ``graph.nbx_system_size`` (this package's dataloaders), else from ``graph.batch``
    (the reference's graphs: arange(B).repeat_interleave(N)), else from a fully-connected edge
    count (E = V (N-1)).  ``fully_connected``: the edge set is every ordered pair of a system."""
    V, E = int(num_nodes), int(num_edges)
    if V == 0:
        raise ValueError("empty graph")
    N = getattr(graph, "nbx_system_size", None)
    batch = getattr(graph, "batch", None)
    if N is not None:
        N = int(N)
    elif batch is not None and batch.numel() == V:
        b = batch.to(device)
        B = int(b.max().item()) + 1
        if V % B or not torch.equal(b, torch.arange(B, device=device).repeat_interleave(V // B)):
            raise NotImplementedError("native models need contiguous systems of equal size")
        N = V // B
    else:
        n = E // V + 1
        if E != V * (n - 1) or V % n:
            raise NotImplementedError("native models need systems of equal size: pass graph.batch for "
                                      "graphs that are not fully connected")
        N = n
    if V % N:
        raise NotImplementedError("native models need systems of equal size")
    B = V // N
    fc = E == V * (N - 1)
    if fc and getattr(graph, "nbx_system_size", None) is None:
        fc = torch.equal(graph.edge_index.to(device), _fc_edge_index_shared(B, N, device))
    return B, N, fc
