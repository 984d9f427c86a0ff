"""numpy restatement of utils/build_fully_connected_graph.py — TEST ORACLE ONLY."""
from __future__ import annotations

import numpy as np


def fc_edge_index(batch_size: int, num_nodes: int) -> np.ndarray:
    """_build_fully_connected_edge_index (build_fully_connected_graph.py:4-20):
    single-system pattern = nonzero(~eye(N)) (row-major over i, then j != i),
    repeated per system with node offsets b*N.  int64 [2, B*N*(N-1)]."""
    ii, jj = np.nonzero(~np.eye(num_nodes, dtype=bool))
    off = np.repeat(np.arange(0, batch_size * num_nodes, num_nodes, dtype=np.int64), ii.size)
    row = np.tile(ii.astype(np.int64), batch_size) + off
    col = np.tile(jj.astype(np.int64), batch_size) + off
    return np.stack([row, col])


def knn_edge_index(loc: np.ndarray, batch_size: int, num_nodes: int, k: int) -> np.ndarray:
    """build_graph_with_knn kNN branch (build_fully_connected_graph.py:42-80):
    per system, cdist, k+1 smallest (ascending), drop the first (self);
    edge_index = [i, neighbour] + system offset.  Ties are unspecified in the
    reference (torch.topk); inputs here are assumed tie-free."""
    loc = loc.reshape(batch_size, num_nodes, -1)
    d = np.sqrt(((loc[:, :, None, :] - loc[:, None, :, :]) ** 2).sum(-1))
    order = np.argsort(d, axis=-1, kind="stable")[:, :, 1:k + 1]
    off = (np.arange(batch_size, dtype=np.int64) * num_nodes)[:, None, None]
    rows = np.broadcast_to(np.arange(num_nodes, dtype=np.int64)[None, :, None], order.shape) + off
    cols = order.astype(np.int64) + off
    return np.stack([rows.reshape(-1), cols.reshape(-1)])


def build_graph_with_knn(loc, batch_size, num_nodes, num_neighbors):
    """build_fully_connected_graph.py:23-40 dispatch (ValueError if k >= N)."""
    num_nodes = int(num_nodes)
    k = num_nodes - 1 if num_neighbors is None else int(num_neighbors)
    if k >= num_nodes:
        raise ValueError("Graph cannot have more neighbors than there are nodes in simulation - 1")
    if k == num_nodes - 1:
        return fc_edge_index(batch_size, num_nodes)
    return knn_edge_index(np.asarray(loc), batch_size, num_nodes, k)
