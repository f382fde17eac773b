"""Graph ingestion on the device: the reference's ``to_undirected`` (PyG 2.4.0 coalesce, reference
data/dataset_handler.py:141) — both directions of every (user, movie) pair, sorted by
row * N + col, duplicates removed — as one HIP radix sort + compaction (lgcn_coalesce_undirected)
instead of a host sort of 2P keys."""
from __future__ import annotations

import ctypes

import torch

from . import _ffi


def to_undirected(edge_index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    """Coalesced undirected edge_index [2, E'] (int64, same device), E' <= 2P."""
    _ffi.require_device(edge_index, "to_undirected")
    if edge_index.dim() != 2 or edge_index.shape[0] != 2:
        raise ValueError(f"edge_index must be [2, P], got {tuple(edge_index.shape)}")
    lib = _ffi.load()
    dev = edge_index.device
    ei = edge_index.to(torch.int64).contiguous()
    P = ei.shape[1]
    N = int(num_nodes)
    nbytes = _ffi._sz(0)
    _ffi.check(lib.lgcn_coalesce_workspace_size(P, N, ctypes.byref(nbytes)), "lgcn_coalesce_workspace_size")
    ws = torch.empty(max(1, nbytes.value), dtype=torch.uint8, device=dev)
    out = torch.empty((2, max(2 * P, 1)), dtype=torch.int64, device=dev)
    cnt = torch.zeros(2, dtype=torch.int64, device=dev)
    _ffi.check(lib.lgcn_coalesce_undirected(ei[0].data_ptr(), ei[1].data_ptr(), P, N, out[0].data_ptr(),
                                            out[1].data_ptr(), cnt.data_ptr(), cnt[1:].data_ptr(), ws.data_ptr(),
                                            ws.numel(), _ffi.stream_of(dev)), "lgcn_coalesce_undirected")
    n, bad = cnt.tolist()
    if bad:
        raise IndexError(f"edge_index holds node ids outside [0, {N})")
    return out[:, :n].contiguous()
