"""Ingestion / split / loader mirror of reference data/dataset_handler.py (CPU)."""
import os

import numpy as np
import pandas as pd
import torch

from data.dataset_handler import (Data, MovieLensDataHandler, build_cluster_loader, to_undirected,
                                  write_synthetic_movielens)
from lgcn_amd import synth
from oracle import lgconv_ref as R


def _handler(tmp_path, users=300, items=150, ratings=6000):
    rp, mp = write_synthetic_movielens(str(tmp_path / "ml"), users, items, ratings, seed=1)
    return MovieLensDataHandler(rp, mp, device=torch.device("cpu")), rp


def test_ids_and_graph_follow_reference_rules(tmp_path):
    h, rp = _handler(tmp_path)
    df = pd.read_csv(rp)
    df = df[df["rating"] >= 4]
    users = list(df["userId"].unique())
    movies = list(df["movieId"].unique())
    assert h.get_num_users_items() == (len(users), len(movies))
    assert [h.user_id_map[u] for u in users] == list(range(len(users)))
    assert [h.movie_id_map[m] for m in movies] == [len(users) + i for i in range(len(movies))]
    u = df["userId"].map(h.user_id_map).values
    m = df["movieId"].map(h.movie_id_map).values
    expect = R.to_undirected(np.vstack([u, m]), h.num_nodes)
    assert np.array_equal(h.edge_index.numpy(), expect)


def test_split_and_persisted_indices(tmp_path, monkeypatch):
    h, _ = _handler(tmp_path)
    monkeypatch.chdir(tmp_path)
    tr, va, te = h.get_datasets(random_state=0)
    E = h.edge_index.shape[1]
    assert tr.edge_index.shape[1] + va.edge_index.shape[1] + te.edge_index.shape[1] == E
    assert abs(tr.edge_index.shape[1] - 0.9 * E) <= 1
    assert os.path.exists("data/indexes/val_indices.npy")
    tr2, va2, te2 = h.get_datasets()  # reload path (train = complement)
    assert torch.equal(tr.edge_index, tr2.edge_index) and torch.equal(va.edge_index, va2.edge_index)
    assert torch.equal(tr.n_id, torch.arange(h.num_nodes))


def test_to_undirected_matches_oracle():
    ei = np.random.default_rng(0).integers(0, 50, (2, 300))
    assert np.array_equal(to_undirected(torch.from_numpy(ei), 50).numpy(), R.to_undirected(ei, 50))


def test_cluster_loader_batches(tmp_path):
    g = synth.bipartite(300, 200, 4000, seed=4)
    ei = torch.from_numpy(g.edge_index)
    loader, part = build_cluster_loader(ei, g.num_nodes, 10, clusters_per_batch=1, shuffle=False)
    sizes = [b.edge_index.shape[1] for b in loader]
    assert len(sizes) == 10 and sum(sizes) == int((part[g.edge_index[0]] == part[g.edge_index[1]]).sum())
    loader3, _ = build_cluster_loader(ei, g.num_nodes, 10, clusters_per_batch=3, shuffle=False, part=part)
    unions = [b.edge_index.shape[1] for b in loader3]
    assert unions == [sum(sizes[0:3]), sum(sizes[3:6]), sum(sizes[6:9]), sizes[9]]
    torch.manual_seed(0)
    first = [b.edge_index.shape[1] for b in build_cluster_loader(ei, g.num_nodes, 10, part=part)[0]]
    assert sorted(first) == sorted(sizes)


def test_data_to_keeps_identity():
    ei = torch.zeros((2, 3), dtype=torch.int64)
    d = Data(edge_index=ei, num_nodes=4)
    assert d.to("cpu") is d and d.edge_index is ei
