"""Cluster-GCN partitions and batches (the reference's ClusterData + DataLoader path).

Reference data/dataset_handler.py:256-288:
    cluster_train = ClusterData(train_dataset, num_parts=100)     # METIS on the train graph
    for cluster in cluster_train:                                # intra-part edges only,
        Data(edge_index=cluster.n_id[cluster.edge_index], ...)   # mapped back to global ids
    DataLoader(train_l, batch_size=1, shuffle=True)
Here: ``partition_nodes`` (liblgcn host partitioner, restreaming LDG instead of METIS) and
``intra_part_edges`` (edges whose endpoints share a part, kept in input order — for a
(row, col)-sorted train set that is the order ClusterData's monotone n_id remap yields).
A batch of q parts is the union of their edge lists (SURVEY.md §7 "Batch semantics"; q = 1 is
the reference).
"""
from __future__ import annotations

import numpy as np

from . import _ffi


def partition_nodes(edge_index, num_nodes: int, num_parts: int, passes: int = 8,
                    imbalance: float = 0.05) -> np.ndarray:
    """part[N] in [0, num_parts): deterministic, balanced on node count. Host-only."""
    ei = np.ascontiguousarray(np.asarray(edge_index if not hasattr(edge_index, "cpu") else edge_index.cpu()),
                              dtype=np.int64)
    src = np.ascontiguousarray(ei[0])
    dst = np.ascontiguousarray(ei[1])
    part = np.empty(num_nodes, dtype=np.int32)
    lib = _ffi.load()
    rc = lib.lgcn_partition_edges(src.ctypes.data, dst.ctypes.data, src.size, num_nodes, num_parts, passes,
                                  float(imbalance), part.ctypes.data)
    if rc != 0:
        raise _ffi.LgcnError(f"lgcn_partition_edges failed (rc={rc}): "
                             f"{lib.lgcn_partition_last_error().decode(errors='replace')}")
    return part


def intra_part_edges(edge_index, part: np.ndarray, num_parts: int) -> list[np.ndarray]:
    """Per part, the [2, E_p] int64 edges with both endpoints in the part (input order kept)."""
    ei = np.asarray(edge_index if not hasattr(edge_index, "cpu") else edge_index.cpu(), dtype=np.int64)
    ps = part[ei[0]]
    keep = np.flatnonzero(ps == part[ei[1]])
    keys = ps[keep]
    order = np.argsort(keys, kind="stable")
    keep = keep[order]
    counts = np.bincount(keys, minlength=num_parts)
    bounds = np.concatenate([[0], np.cumsum(counts)])
    sel = ei[:, keep]
    return [np.ascontiguousarray(sel[:, bounds[p]:bounds[p + 1]]) for p in range(num_parts)]


def intra_fraction(edge_index, part: np.ndarray) -> float:
    ei = np.asarray(edge_index if not hasattr(edge_index, "cpu") else edge_index.cpu())
    if ei.shape[1] == 0:
        return 1.0
    return float(np.mean(part[ei[0]] == part[ei[1]]))


def part_sizes(part: np.ndarray, num_parts: int) -> np.ndarray:
    return np.bincount(part, minlength=num_parts)


def cluster_batches(train_edge_index, num_nodes: int, num_parts: int, parts_per_batch: int,
                    order_seed: int = 1) -> tuple[np.ndarray, float, list[np.ndarray]]:
    """The C3/C4 batches: partition the train graph into ``num_parts`` parts, then union the
    intra-part edges of ``parts_per_batch`` parts per batch, parts taken in a seeded permutation
    (reference data/dataset_handler.py:273-285 with q parts per DataLoader item).
    Returns (part[N], intra-part edge fraction, list of [2, E_b] int64 batch edge lists)."""
    part = partition_nodes(train_edge_index, num_nodes, num_parts)
    f_intra = intra_fraction(train_edge_index, part)
    lists = intra_part_edges(train_edge_index, part, num_parts)
    order = np.random.default_rng(order_seed).permutation(num_parts)
    batches = [np.ascontiguousarray(np.concatenate([lists[p] for p in order[b:b + parts_per_batch]], axis=1))
               for b in range(0, num_parts, parts_per_batch)]
    return part, f_intra, batches
