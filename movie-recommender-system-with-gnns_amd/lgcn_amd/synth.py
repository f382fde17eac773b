"""Synthetic MovieLens-shaped bipartite graphs (no dataset exists offline).

The reference builds its graph from MovieLens-25M ratings >= 4 (reference
data/dataset_handler.py:105-141): users are ids [0, U), movies [U, U+I), and
``to_undirected`` makes both directions and coalesces (sorted by row*N+col, deduplicated).
``ml25m_shaped`` produces the same structure from seeded Zipf-like user activity and item
popularity, calibrated to ML-25M's scale (U=162,541, I=59,047, ~12.45M unique rating>=4 pairs,
E ≈ 2.49e7 directed edges) and skew (hub items with 1e4–1e5 raters, medians of tens).
"""
from __future__ import annotations

import dataclasses

import numpy as np

ML25M_USERS = 162_541
ML25M_ITEMS = 59_047
ML25M_PAIRS = 12_450_000


@dataclasses.dataclass
class BipartiteGraph:
    num_users: int
    num_items: int
    edge_index: np.ndarray  # int64 [2, E], coalesced undirected (users first)

    @property
    def num_nodes(self) -> int:
        return self.num_users + self.num_items

    @property
    def num_edges(self) -> int:
        return int(self.edge_index.shape[1])

    def degree_stats(self) -> dict:
        deg = np.bincount(self.edge_index[1], minlength=self.num_nodes)
        du, di = deg[: self.num_users], deg[self.num_users:]
        return {"user_max": int(du.max()), "user_median": float(np.median(du)),
                "item_max": int(di.max()), "item_median": float(np.median(di))}


def zipf_weights(n: int, alpha: float, offset: float, rng: np.random.Generator) -> np.ndarray:
    w = 1.0 / np.power(np.arange(1, n + 1, dtype=np.float64) + offset, alpha)
    w = w[rng.permutation(n)]  # hubs at random ids, as in real id maps
    return w / w.sum()


def undirected_from_pairs(users: np.ndarray, items: np.ndarray, num_users: int, num_items: int) -> np.ndarray:
    """Coalesced undirected edge_index of user–item pairs (reference data/dataset_handler.py:139-141)."""
    N = num_users + num_items
    u = users.astype(np.int64)
    i = items.astype(np.int64) + num_users
    key = np.concatenate([u * N + i, i * N + u])
    key = np.unique(key)
    return np.stack([key // N, key % N])


def random_pairs(num_users: int, num_items: int, num_pairs: int, seed: int = 0, user_alpha: float = 0.75,
                 user_offset: float = 40.0, item_alpha: float = 1.0, item_offset: float = 12.0):
    rng = np.random.default_rng(seed)
    max_pairs = num_users * num_items
    num_pairs = min(num_pairs, max_pairs)
    pu = zipf_weights(num_users, user_alpha, user_offset, rng)
    pi = zipf_weights(num_items, item_alpha, item_offset, rng)
    keys = np.empty(0, dtype=np.int64)
    draw = int(num_pairs * 1.25) + 16
    for _ in range(12):
        u = rng.choice(num_users, size=draw, p=pu)
        it = rng.choice(num_items, size=draw, p=pi)
        keys = np.unique(np.concatenate([keys, u.astype(np.int64) * num_items + it]))
        if keys.size >= num_pairs:
            break
        draw = int((num_pairs - keys.size) * 2.0) + 1024
    if keys.size > num_pairs:
        keys = np.sort(rng.choice(keys, size=num_pairs, replace=False))
    return keys // num_items, keys % num_items


def bipartite(num_users: int, num_items: int, num_pairs: int, seed: int = 0, **kw) -> BipartiteGraph:
    u, i = random_pairs(num_users, num_items, num_pairs, seed, **kw)
    return BipartiteGraph(num_users, num_items, undirected_from_pairs(u, i, num_users, num_items))


# user-activity skew of the ML-25M-shaped graph: calibrated so the heaviest user holds ~3e4
# rating>=4 pairs (seed 0: user max 31,703, median 35; item max 58,571, median 62)
ML25M_USER_ALPHA = 0.82
ML25M_USER_OFFSET = 2.0


def ml25m_shaped(seed: int = 0, scale: float = 1.0) -> BipartiteGraph:
    """The C2 graph (scale=1): ML-25M-shaped, E ≈ 2.49e7 directed edges."""
    U = max(2, int(ML25M_USERS * scale))
    I = max(2, int(ML25M_ITEMS * scale))
    P = max(1, int(ML25M_PAIRS * scale))
    return bipartite(U, I, P, seed, user_alpha=ML25M_USER_ALPHA, user_offset=ML25M_USER_OFFSET)


def train_split(edge_index: np.ndarray, frac: float = 0.9, seed: int = 0) -> np.ndarray:
    """The train share of the directed edges, kept in coalesced order (reference
    data/dataset_handler.py:160-199: a seeded permutation of edge positions, indices sorted)."""
    E = edge_index.shape[1]
    perm = np.random.default_rng(seed).permutation(E)
    return np.ascontiguousarray(edge_index[:, np.sort(perm[:int(frac * E)])])


def planted_bipartite(num_users: int, num_items: int, communities: int, degree: int = 20, p_in: float = 0.8,
                      seed: int = 0) -> tuple[BipartiteGraph, np.ndarray]:
    """A user–item graph with planted taste communities, for judging the partitioner (the
    reference's METIS has no stand-in here): user u belongs to a random community, item i to
    community i % k; each of a user's `degree` draws is an item of its own community with
    probability p_in, else a uniform item. Returns (graph, ground-truth community per node)."""
    rng = np.random.default_rng(seed)
    k = communities
    cu = rng.integers(0, k, num_users)
    u = np.repeat(np.arange(num_users, dtype=np.int64), degree)
    inside = rng.random(u.size) < p_in
    it = rng.integers(0, num_items, u.size)
    sel = np.flatnonzero(inside)
    it[sel] = cu[u[sel]] + k * rng.integers(0, num_items // k, sel.size)
    g = BipartiteGraph(num_users, num_items, undirected_from_pairs(u, it, num_users, num_items))
    return g, np.concatenate([cu, np.arange(num_items) % k]).astype(np.int32)


def planted_ml25m(communities: int = 1024, p_in: float = 0.8, scale: float = 1.0,
                  seed: int = 0) -> tuple[BipartiteGraph, np.ndarray]:
    """An ML-25M-sized graph (the C2 users, items, pair count and user-activity skew) with planted
    taste communities, for judging the partitioner at C3 scale: user u is in a random community,
    item i in community i % k; each of u's draws (Zipf-skewed activity, as ``ml25m_shaped``) is,
    with probability p_in, a uniform item of u's community, else an item by global Zipf
    popularity. Up to P pairs: heavy users saturate their community's items, and the draw stops
    after 12 rounds (full scale: 12,447,700 of 12,450,000). Returns (graph, ground-truth
    community per node)."""
    rng = np.random.default_rng(seed)
    U = max(2, int(ML25M_USERS * scale))
    I = max(2, int(ML25M_ITEMS * scale))
    P = max(1, int(ML25M_PAIRS * scale))
    k = communities
    cu = rng.integers(0, k, U)
    pu = zipf_weights(U, ML25M_USER_ALPHA, ML25M_USER_OFFSET, rng)
    pi = zipf_weights(I, 1.0, 12.0, rng)
    per = np.bincount(np.arange(I) % k, minlength=k)  # items per community
    keys = np.empty(0, dtype=np.int64)
    draw = int(P * 1.3) + 16
    for _ in range(12):
        u = rng.choice(U, size=draw, p=pu)
        it = rng.choice(I, size=draw, p=pi)
        inside = rng.random(draw) < p_in
        c = cu[u[inside]]
        it[inside] = c + k * (rng.random(int(inside.sum())) * per[c]).astype(np.int64)
        keys = np.unique(np.concatenate([keys, u.astype(np.int64) * I + it]))
        if keys.size >= P:
            break
        draw = int((P - keys.size) * 2.0) + 1024
    if keys.size > P:
        keys = np.sort(rng.choice(keys, size=P, replace=False))
    g = BipartiteGraph(U, I, undirected_from_pairs(keys // I, keys % I, U, I))
    return g, np.concatenate([cu, np.arange(I) % k]).astype(np.int32)


def bipartite_device(num_users: int, num_items: int, num_pairs: int, seed: int = 0, device="cuda",
                     user_alpha: float = 0.75, user_offset: float = 40.0, item_alpha: float = 1.0,
                     item_offset: float = 12.0):
    """The same Zipf-like user/item draw as ``random_pairs`` but generated on the device with torch
    (for C5-sized graphs: 5e8 edges would need tens of GB of host RAM in numpy). Returns the
    coalesced undirected edge_index [2, E] (int64, on ``device``). Not bit-identical to the numpy
    generator (different RNG); seeded and deterministic for a given device type."""
    import torch

    dev = torch.device(device)
    g = torch.Generator(device=dev).manual_seed(seed)

    def weights(n, alpha, offset):
        w = 1.0 / torch.pow(torch.arange(1, n + 1, device=dev, dtype=torch.float64) + offset, alpha)
        w = w[torch.randperm(n, device=dev, generator=g)]
        return (w / w.sum()).to(torch.float32)

    pu = weights(num_users, user_alpha, user_offset)
    pi = weights(num_items, item_alpha, item_offset)
    cu = torch.cumsum(pu.double(), 0)
    ci = torch.cumsum(pi.double(), 0)
    keys = torch.empty(0, dtype=torch.int64, device=dev)
    draw = int(num_pairs * 1.3) + 1024
    for _ in range(12):
        ru = torch.rand(draw, device=dev, generator=g, dtype=torch.float64) * cu[-1]
        ri = torch.rand(draw, device=dev, generator=g, dtype=torch.float64) * ci[-1]
        u = torch.searchsorted(cu, ru).clamp_(max=num_users - 1)
        it = torch.searchsorted(ci, ri).clamp_(max=num_items - 1)
        del ru, ri
        keys = torch.unique(torch.cat([keys, u * num_items + it]))
        del u, it
        if keys.numel() >= num_pairs:
            break
        draw = int((num_pairs - keys.numel()) * 2.0) + 1024
    if keys.numel() > num_pairs:
        pick = torch.randperm(keys.numel(), device=dev, generator=g)[:num_pairs]
        keys = torch.sort(keys[pick]).values
    N = num_users + num_items
    users = keys // num_items
    items = keys % num_items + num_users
    del keys
    key = torch.cat([users * N + items, items * N + users])
    del users, items
    key = torch.sort(key).values  # unique already: (u, i) pairs are distinct and directions disjoint
    return torch.stack([key // N, key % N])


C5_USERS = 10_000_000
C5_ITEMS = 1_000_000
C5_PAIRS = 250_000_000
