"""Synthetic MovieLens-shaped graph generator (bench / tests input) — CPU."""
import numpy as np

from lgcn_amd import synth


def test_bipartite_is_coalesced_undirected():
    g = synth.bipartite(500, 300, 5000, seed=0)
    ei = g.edge_index
    N = g.num_nodes
    key = ei[0] * N + ei[1]
    assert np.all(np.diff(key) > 0)  # sorted by row*N+col, no duplicates
    rev = np.sort(ei[1] * N + ei[0])
    assert np.array_equal(rev, key)  # symmetric
    assert np.all((ei[0] < 500) != (ei[1] < 500))  # every edge joins a user and an item
    assert g.num_edges == 2 * 5000


def test_seeded_and_skewed():
    a = synth.bipartite(2000, 500, 20000, seed=3)
    b = synth.bipartite(2000, 500, 20000, seed=3)
    assert np.array_equal(a.edge_index, b.edge_index)
    s = a.degree_stats()
    assert s["item_max"] > 10 * s["item_median"]


def test_ml25m_scaled_shape():
    g = synth.ml25m_shaped(seed=0, scale=0.01)
    assert g.num_users == int(162_541 * 0.01) and g.num_items == int(59_047 * 0.01)
    assert g.num_edges == 2 * int(12_450_000 * 0.01)
