"""ORACLE — test infrastructure, not product code.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.

The reference's propagation restated with the exact torch primitives PyG 2.4.0 executes for
``LGConv()(x, edge_index)`` on a plain edge_index tensor (environment.yml:24; call site
reference models/light_gcn.py:33):

    gcn_norm:  deg = zeros(N).scatter_add_(0, col, ones(E)); dis = deg.pow_(-0.5);
               dis.masked_fill_(dis == inf, 0); w = dis[row] * ones * dis[col]
    propagate: x_j = x.index_select(0, row); msg = w.view(-1, 1) * x_j;
               out = x.new_zeros(N, d).scatter_add_(0, col.view(-1,1).expand_as(msg), msg)

and the reference LightGCN module around it (models/light_gcn.py:13-64), so the reference's
own harness (utils/train_test.py) can be driven on CPU with it. On CPU these are the
reference's own arithmetic (deterministic scatter_add_); this is also the "reference CPU path"
that bench.py times as cpu_baseline.
"""
from __future__ import annotations

import warnings

import torch
import torch.nn as nn


def gcn_norm_torch(edge_index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    row, col = edge_index[0], edge_index[1]
    ew = torch.ones(edge_index.size(1), dtype=torch.float32, device=edge_index.device)
    deg = torch.zeros(num_nodes, dtype=torch.float32, device=edge_index.device).scatter_add_(0, col, ew)
    dis = deg.pow_(-0.5)
    dis.masked_fill_(dis == float("inf"), 0)
    return dis[row] * ew * dis[col]


def lgconv_torch(x: torch.Tensor, edge_index: torch.Tensor, w: torch.Tensor | None = None) -> torch.Tensor:
    if w is None:
        w = gcn_norm_torch(edge_index, x.size(0))
    x_j = x.index_select(0, edge_index[0])
    msg = w.view(-1, 1) * x_j
    idx = edge_index[1].view(-1, 1).expand_as(msg)
    return x.new_zeros(x.shape).scatter_add_(0, idx, msg)


class OracleLGConv(nn.Module):
    def forward(self, x, edge_index):
        return lgconv_torch(x, edge_index)


class OracleLightGCN(nn.Module):
    """CPU restatement of reference models/light_gcn.py:13-64 on the torch-primitive LGConv."""

    def __init__(self, num_users, num_items, num_layers=4, dim_h=64):
        super().__init__()
        self.num_users = num_users
        self.num_items = num_items
        self.num_layers = num_layers
        self.dim_h = dim_h
        self.user_embedding = nn.Embedding(num_embeddings=num_users, embedding_dim=dim_h)
        self.item_embedding = nn.Embedding(num_embeddings=num_items, embedding_dim=dim_h)
        self.convs = nn.ModuleList(OracleLGConv() for _ in range(num_layers))
        nn.init.normal_(self.user_embedding.weight, std=0.01)
        nn.init.normal_(self.item_embedding.weight, std=0.01)

    def forward(self, edge_index):
        emb = torch.cat([self.user_embedding.weight, self.item_embedding.weight])
        embs = [emb]
        for conv in self.convs:
            emb = conv(emb, edge_index)
            embs.append(emb)
        emb_final = 1 / (self.num_layers + 1) * torch.mean(torch.stack(embs, dim=1), dim=1)
        return torch.split(emb_final, [self.num_users, self.num_items])

    def get_embeddings(self, user_indices=None, item_indices=None):
        if user_indices is not None and item_indices is not None:
            return self.user_embedding.weight[user_indices], self.item_embedding.weight[item_indices]
        if user_indices is not None:
            return self.user_embedding.weight[user_indices], None
        if item_indices is not None:
            return None, self.item_embedding.weight[item_indices]
        warnings.warn("Both indices not provided", UserWarning)
        return None, None


def time_reference_forward(user_w: torch.Tensor, item_w: torch.Tensor, edge_index: torch.Tensor, K: int,
                           reps: int = 3, warmup: bool = True) -> float:
    """Median seconds of the reference CPU op sequence for one K-layer forward (no autograd),
    including gcn_norm per layer exactly as LGConv does. warmup=False times the
    first run too (for multi-second forwards, where one untimed run would double the cost)."""
    import time

    times = []
    with torch.no_grad():
        for _ in range(reps + (1 if warmup else 0)):
            t0 = time.perf_counter()
            emb = torch.cat([user_w, item_w])
            embs = [emb]
            for _ in range(K):
                emb = lgconv_torch(emb, edge_index)
                embs.append(emb)
            out = 1 / (K + 1) * torch.mean(torch.stack(embs, dim=1), dim=1)
            torch.split(out, [user_w.shape[0], item_w.shape[0]])
            times.append(time.perf_counter() - t0)
    times = sorted(times[1:] if warmup else times)
    return times[len(times) // 2]


def time_csr_forward(user_w: torch.Tensor, item_w: torch.Tensor, edge_index: torch.Tensor, K: int,
                     reps: int = 3) -> float:
    """Median seconds of a K-layer forward with the "torch_sparse-style" CPU SpMM: the same
    gcn_norm-weighted adjacency as one CSR matrix (built once, outside the timing, as
    torch_sparse's SparseTensor would be), then y = torch.sparse.mm(A, x) per layer and the
    layer-stack mean (BASELINE.md §3's second CPU baseline)."""
    import time

    N = user_w.shape[0] + item_w.shape[0]
    w = gcn_norm_torch(edge_index, N)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", UserWarning)  # "sparse CSR support is in beta"
        A = torch.sparse_coo_tensor(torch.stack([edge_index[1], edge_index[0]]), w, (N, N)).coalesce().to_sparse_csr()
    times = []
    with torch.no_grad():
        for _ in range(reps + 1):
            t0 = time.perf_counter()
            emb = torch.cat([user_w, item_w])
            acc = emb.clone()
            for _ in range(K):
                emb = torch.sparse.mm(A, emb)
                acc += emb
            out = acc / (K + 1) * (1 / (K + 1))
            torch.split(out, [user_w.shape[0], item_w.shape[0]])
            times.append(time.perf_counter() - t0)
    times = sorted(times[1:])
    return times[len(times) // 2]
