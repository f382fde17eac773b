"""Seeded test graphs shared by the CPU and GPU suites (reference-shaped edge sets)."""
from __future__ import annotations

import numpy as np

from lgcn_amd import synth


def toy():
    """The reference's own smoke graph: models/light_gcn.py:68-73 (10 users, 15 items, 20 edges)."""
    ei = np.array([list(range(20)), list(range(10, 20)) + list(range(10))], dtype=np.int64)
    return 10, 15, ei


def sym(U=300, I=200, pairs=3000, seed=0):
    g = synth.bipartite(U, I, pairs, seed)
    return U, I, g.edge_index


def subsampled(U=300, I=200, pairs=3000, frac=0.9, seed=0):
    """A random directed-edge subset as the reference's split makes: asymmetric,
    with nodes that keep out-edges but lose every in-edge (weight 0)."""
    U, I, ei = sym(U, I, pairs, seed)
    rng = np.random.default_rng(seed + 100)
    keep = np.sort(rng.choice(ei.shape[1], int(frac * ei.shape[1]), replace=False))
    return U, I, np.ascontiguousarray(ei[:, keep])


def shuffled(U=300, I=200, pairs=3000, seed=0):
    """Unsorted input (e.g. a union of cluster edge lists)."""
    U, I, ei = subsampled(U, I, pairs, 0.7, seed)
    rng = np.random.default_rng(seed + 7)
    return U, I, np.ascontiguousarray(ei[:, rng.permutation(ei.shape[1])])


def hub(U=2000, I=50, seed=0):
    """Heavy skew: one item rated by every user (in-degree U), so rows split into many chunks."""
    rng = np.random.default_rng(seed)
    users = np.concatenate([np.arange(U), rng.integers(0, U, 3 * U)])
    items = np.concatenate([np.zeros(U, np.int64), rng.integers(1, I, 3 * U)])
    ei = synth.undirected_from_pairs(users, items, U, I)
    return U, I, ei


def with_isolated(U=100, I=80, seed=0):
    """Users and items that appear in no edge (zero rows everywhere)."""
    rng = np.random.default_rng(seed)
    users = rng.integers(0, U // 2, 400)
    items = rng.integers(0, I // 2, 400)
    return U, I, synth.undirected_from_pairs(users, items, U, I)


def embeddings(U, I, d, seed=0):
    rng = np.random.default_rng(seed)
    uw = (rng.standard_normal((U, d)) * 0.01).astype(np.float32)
    iw = (rng.standard_normal((I, d)) * 0.01).astype(np.float32)
    return uw, iw


ALL = {"toy": toy, "sym": sym, "subsampled": subsampled, "shuffled": shuffled, "hub": hub,
       "isolated": with_isolated}
