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


def test_train_split_keeps_coalesced_order():
    g = synth.bipartite(400, 200, 4000, seed=1)
    tr = synth.train_split(g.edge_index, 0.9, seed=0)
    assert tr.shape[1] == int(0.9 * g.num_edges)
    N = g.num_nodes
    key = tr[0] * N + tr[1]
    assert np.all(np.diff(key) > 0)  # still (row, col)-sorted, a subset of the coalesced list
    assert np.isin(key, g.edge_index[0] * N + g.edge_index[1]).all()
    assert np.array_equal(tr, synth.train_split(g.edge_index, 0.9, seed=0))


def test_planted_ml25m_small_scale():
    g, truth = synth.planted_ml25m(64, scale=0.01, seed=2)
    assert g.num_users == int(162_541 * 0.01) and g.num_items == int(59_047 * 0.01)
    # the community-local draws saturate small communities, so the pair count can fall short of P
    assert 0.9 * 2 * int(12_450_000 * 0.01) <= g.num_edges <= 2 * int(12_450_000 * 0.01)
    ei = g.edge_index
    assert np.all((ei[0] < g.num_users) != (ei[1] < g.num_users))
    assert truth.shape == (g.num_nodes,) and truth.max() < 64
    # far more pairs inside the planted communities than chance (1/64); at this scale a community
    # holds ~9 items, so heavy users saturate it and deduplication drops most inside draws
    assert np.mean(truth[ei[0]] == truth[ei[1]]) > 0.1
