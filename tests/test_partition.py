"""Host partitioner (METIS replacement) and Cluster-GCN batching — no GPU needed."""
import numpy as np
import pytest

from lgcn_amd import _ffi, cluster, synth


def planted(k=8, per=50, p_in=0.3, p_out=0.005, seed=0):
    """Undirected graph with k planted communities."""
    rng = np.random.default_rng(seed)
    n = k * per
    blocks = np.repeat(np.arange(k), per)
    a = rng.random((n, n)) < np.where(blocks[:, None] == blocks[None, :], p_in, p_out)
    a = np.triu(a, 1)
    r, c = np.nonzero(a)
    key = np.unique(np.concatenate([r * n + c, c * n + r]))
    return n, np.stack([key // n, key % n])


def test_partition_is_deterministic_and_balanced():
    g = synth.bipartite(400, 300, 6000, seed=2)
    for k in (1, 2, 7, 64):
        a = cluster.partition_nodes(g.edge_index, g.num_nodes, k)
        b = cluster.partition_nodes(g.edge_index, g.num_nodes, k)
        assert np.array_equal(a, b)
        assert a.min() >= 0 and a.max() < k
        sizes = cluster.part_sizes(a, k)
        assert sizes.max() - sizes.min() <= 1 and sizes.sum() == g.num_nodes


def test_partition_finds_planted_communities():
    n, ei = planted()
    part = cluster.partition_nodes(ei, n, 8)
    rnd = np.random.default_rng(0).integers(0, 8, n)
    assert cluster.intra_fraction(ei, part) > 0.6
    assert cluster.intra_fraction(ei, part) > 3 * cluster.intra_fraction(ei, rnd)


def test_partition_beats_random_on_ml25m_shaped():
    g = synth.ml25m_shaped(seed=0, scale=0.02)
    part = cluster.partition_nodes(g.edge_index, g.num_nodes, 16)
    rnd = np.random.default_rng(0).integers(0, 16, g.num_nodes)
    assert cluster.intra_fraction(g.edge_index, part) > 1.5 * cluster.intra_fraction(g.edge_index, rnd)


def test_intra_part_edges_order_and_coverage():
    g = synth.bipartite(200, 100, 2000, seed=3)
    ei = g.edge_index
    part = cluster.partition_nodes(ei, g.num_nodes, 5)
    lists = cluster.intra_part_edges(ei, part, 5)
    keep = part[ei[0]] == part[ei[1]]
    assert sum(x.shape[1] for x in lists) == int(keep.sum())
    pos = {(int(a), int(b)): i for i, (a, b) in enumerate(ei.T)}
    for p, x in enumerate(lists):
        assert np.all(part[x[0]] == p) and np.all(part[x[1]] == p)
        idx = [pos[(int(a), int(b))] for a, b in x.T]
        assert idx == sorted(idx)  # input (row, col) order kept, as ClusterData's monotone remap


def test_partition_rejects_bad_ids():
    with pytest.raises(_ffi.LgcnError):
        cluster.partition_nodes(np.array([[0, 5], [1, 0]]), 3, 2)


def test_empty_and_tiny():
    part = cluster.partition_nodes(np.zeros((2, 0), np.int64), 5, 3)
    assert sorted(cluster.part_sizes(part, 3).tolist()) == [1, 2, 2]
    assert cluster.intra_fraction(np.zeros((2, 0), np.int64), part) == 1.0


def test_partition_recovers_planted_bipartite_communities():
    """Refined partition (LDG passes + size-constrained label propagation + min-loss balance
    fix-up) keeps >= 0.9 of the ground truth's intra-part edges on a planted user-item graph;
    measured 0.757 vs 0.778 (tools/partition_quality.py has the larger case: 0.756 vs 0.781;
    plain 4-pass LDG with the old fix-up reached 0.655 there)."""
    g, truth = synth.planted_bipartite(8000, 3200, 64, seed=1)
    part = cluster.partition_nodes(g.edge_index, g.num_nodes, 64)
    sizes = cluster.part_sizes(part, 64)
    assert sizes.max() - sizes.min() <= 1
    q, t = cluster.intra_fraction(g.edge_index, part), cluster.intra_fraction(g.edge_index, truth)
    assert q >= 0.9 * t, (q, t)


def test_cluster_batches_union_of_parts():
    """cluster_batches: every batch is the union of parts_per_batch parts' intra-part edges, every
    intra-part edge lands in exactly one batch, in the parts' seeded order."""
    from lgcn_amd import cluster, synth

    g = synth.bipartite(600, 300, 6000, seed=4)
    part, f, batches = cluster.cluster_batches(g.edge_index, g.num_nodes, 16, 4)
    assert len(batches) == 4 and 0 < f < 1
    lists = cluster.intra_part_edges(g.edge_index, part, 16)
    order = np.random.default_rng(1).permutation(16)
    for b, ei in enumerate(batches):
        want = np.concatenate([lists[p] for p in order[4 * b:4 * b + 4]], axis=1)
        assert np.array_equal(ei, want)
    assert sum(b.shape[1] for b in batches) == int(round(f * g.num_edges))
