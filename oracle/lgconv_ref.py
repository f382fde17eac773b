"""ORACLE — test infrastructure, not product code.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker. The product path (lgcn_amd, models/, utils/) never calls it.

CPU restatement (numpy, fp32) of the reference's hot path, step by step:

  * to_undirected / coalesce (PyG 2.4.0 utils/undirected.py, called at reference
    data/dataset_handler.py:141): concat (row,col),(col,row), sort by row*N+col, dedupe.
  * gcn_norm(add_self_loops=False) (PyG 2.4.0 nn/conv/gcn_conv.py, reached from LGConv.forward
    at reference models/light_gcn.py:33): deg = fp32 scatter-sum of ones at edge_index[1],
    dis = deg^-1/2 (1/sqrt, inf -> 0), w = (dis[row] * 1) * dis[col].
  * LGConv.propagate (PyG 2.4.0 nn/conv/message_passing.py + utils/scatter.py):
    x_j = x[edge_index[0]], msg = w[:,None] * x_j, out = zeros.scatter_add_(0, edge_index[1], msg)
    — np.add.at adds sequentially in edge order, as CPU scatter_add_ does.
  * LightGCN.forward (reference models/light_gcn.py:28-40):
    out = (sum(stack([x0..xK])) / (K+1)) * fp32(1/(K+1)), split [U, I]   
  * the analytic gradient of the same (what autograd computes through index_select /
    mul / scatter_add_ / stack / mean / mul).

PyG 2.4.0 (environment.yml:24) is not installed here and not vendored in the reference; its
published algorithm is restated above and pinned by tests/golden (see tests/golden/make_golden.py
and DESIGN.md §Oracle for what each fixture is anchored on).
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


def to_undirected(edge_index: np.ndarray, num_nodes: int) -> np.ndarray:
    """PyG to_undirected on an unweighted edge_index: both directions, coalesced (sorted by
    row*N+col, duplicates removed)."""
    row, col = edge_index
    r = np.concatenate([row, col]).astype(np.int64)
    c = np.concatenate([col, row]).astype(np.int64)
    key = np.unique(r * num_nodes + c)
    return np.stack([key // num_nodes, key % num_nodes])


def in_degree_f32(edge_index: np.ndarray, num_nodes: int) -> np.ndarray:
    """scatter(ones, edge_index[1], reduce='sum') in fp32 — exact below 2^24 (then saturating,
    as a sequential fp32 sum of ones does)."""
    cnt = np.bincount(edge_index[1], minlength=num_nodes).astype(np.int64)
    return np.minimum(cnt, 1 << 24).astype(F32)


def inv_sqrt_deg(deg: np.ndarray) -> np.ndarray:
    with np.errstate(divide="ignore"):
        dis = (F32(1.0) / np.sqrt(deg.astype(F32))).astype(F32)
    dis[np.isinf(dis)] = F32(0.0)
    return dis


def gcn_norm(edge_index: np.ndarray, num_nodes: int) -> np.ndarray:
    """Edge weights in edge order (PyG 2.4.0 gcn_norm, add_self_loops=False)."""
    dis = inv_sqrt_deg(in_degree_f32(edge_index, num_nodes))
    row, col = edge_index
    return ((dis[row] * F32(1.0)) * dis[col]).astype(F32)


def lgconv(x: np.ndarray, edge_index: np.ndarray, w: np.ndarray | None = None) -> np.ndarray:
    """One LGConv layer: out[i] = sum_{e: col_e = i} w_e * x[row_e], added in edge order."""
    x = np.asarray(x, dtype=F32)
    N = x.shape[0]
    if w is None:
        w = gcn_norm(edge_index, N)
    row, col = edge_index
    msg = (w[:, None].astype(F32) * x[row]).astype(F32)
    out = np.zeros_like(x)
    np.add.at(out, col, msg)
    return out


def lgconv_transposed(dy: np.ndarray, edge_index: np.ndarray, w: np.ndarray) -> np.ndarray:
    """Autograd of lgconv w.r.t. x: dx[j] = sum_{e: row_e = j} w_e * dy[col_e] in edge order
    (gather -> mul -> index_add_)."""
    row, col = edge_index
    g = (dy[col] * w[:, None]).astype(F32)
    out = np.zeros_like(dy)
    np.add.at(out, row, g)
    return out


def lightgcn_forward(user_w: np.ndarray, item_w: np.ndarray, edge_index: np.ndarray, K: int):
    x0 = np.concatenate([user_w, item_w]).astype(F32)
    N = x0.shape[0]
    w = gcn_norm(edge_index, N)
    embs = [x0]
    x = x0
    for _ in range(K):
        x = lgconv(x, edge_index, w)
        embs.append(x)
    s = embs[0].copy()
    for e in embs[1:]:
        s = (s + e).astype(F32)
    out = ((s / F32(K + 1)).astype(F32) * F32(1.0 / (K + 1))).astype(F32)
    U = user_w.shape[0]
    return out[:U], out[U:]


def lightgcn_backward(dout: np.ndarray, edge_index: np.ndarray, U: int, K: int):
    """(grad_user, grad_item) for out = lightgcn_forward(...) given dout [N, d]."""
    dout = np.asarray(dout, dtype=F32)
    N = dout.shape[0]
    w = gcn_norm(edge_index, N)
    g = ((dout * F32(1.0 / (K + 1))).astype(F32) / F32(K + 1)).astype(F32)
    G = g
    for _ in range(K):
        G = (g + lgconv_transposed(G, edge_index, w)).astype(F32)
    return G[:U], G[U:]


def csr_by_key(key: np.ndarray, other: np.ndarray, num_nodes: int):
    """Stable grouping of edges by key: (rowptr int64[N+1], col int32[E], eid int32[E])."""
    key = np.asarray(key, dtype=np.int64)
    perm = np.argsort(key, kind="stable")
    cnt = np.bincount(key, minlength=num_nodes)
    rowptr = np.zeros(num_nodes + 1, dtype=np.int64)
    np.cumsum(cnt, out=rowptr[1:])
    return rowptr, np.asarray(other, dtype=np.int64)[perm].astype(np.int32), perm.astype(np.int32)


def csr_values(rowptr: np.ndarray, col: np.ndarray, dis: np.ndarray) -> np.ndarray:
    rows = np.repeat(np.arange(len(rowptr) - 1), np.diff(rowptr))
    return (dis[rows] * dis[col]).astype(F32)


# ---- reference harness restatements (utils/train_test.py, utils/helpers.py) ----

def bpr_loss_np(eu_f, eu, ep_f, ep, en_f, en, bpr_coeff=5e-3) -> float:
    """float64 restatement of reference utils/train_test.py:18-51 (for tolerance checks)."""
    f = lambda a: np.asarray(a, dtype=np.float64)
    eu_f, eu, ep_f, ep, en_f, en = map(f, (eu_f, eu, ep_f, ep, en_f, en))
    reg = bpr_coeff * (eu * eu + ep * ep + en * en).mean()
    n = lambda a: a / np.linalg.norm(a, axis=1, keepdims=True)
    cp = (n(eu_f) * n(ep_f)).sum(1)
    cn = (n(eu_f) * n(en_f)).sum(1)
    z = 10 * (cp - cn)
    sp = np.logaddexp(0.0, z)
    return float(-sp.mean() / 10.0 + reg)
