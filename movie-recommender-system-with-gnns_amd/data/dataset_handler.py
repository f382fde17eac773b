"""MovieLens ingestion, split and Cluster-GCN loader with the reference's API
(reference data/dataset_handler.py:66-298, class MovieLensDataHandler).

Kept from the reference: ratings.csv / movies.csv schema; rating >= 4 filter (:106); user ids
[0, U) and movie ids [U, U+I) in order of first appearance (:115-118); ``to_undirected``
coalesce (:141); 90/5/5 random split over the DIRECTED edge positions with sorted index lists
persisted as data/indexes/{val,test}_indices.npy and train = the complement (:144-253);
``get_data_training`` returning (train loader over Cluster-GCN parts, val Data, test Data)
(:256-288); ``get_num_users_items`` (:290-298).
Different by necessity: no HTTP download (:16-64; no network — a missing file raises); the
partition comes from lgcn_amd.cluster (host LDG partitioner) instead of METIS/ClusterData;
``Data`` below is the minimal stand-in for torch_geometric.data.Data that the harness needs.
Optional extras: ``random_state`` for a reproducible split (the reference's is unseeded, Q8),
``clusters_per_batch`` for Cluster-GCN multi-part batches (union of edge lists).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

import numpy as np
import pandas as pd
import torch

from lgcn_amd import cluster as _cluster

MOVIELENS_25M_URL = "https://files.grouplens.org/datasets/movielens/ml-25m.zip"
DATA_DIR = "data/movielens-25m"

torch.manual_seed(0)  # import-time seeding, as reference data/dataset_handler.py:20-24
torch.cuda.manual_seed(0)
torch.cuda.manual_seed_all(0)


class Data:
    """Minimal graph record: ``edge_index`` (LongTensor [2, E], global ids), ``num_nodes`` and
    optional ``n_id``; ``.to(device)`` moves every tensor attribute."""

    def __init__(self, edge_index: Optional[torch.Tensor] = None, num_nodes: Optional[int] = None, **attrs):
        self.edge_index = edge_index
        self.num_nodes = num_nodes
        for k, v in attrs.items():
            setattr(self, k, v)

    def to(self, device) -> "Data":
        """Moves tensor attributes in place and returns self (as PyG's Data.to). A tensor already
        on ``device`` stays the same object, so its cached propagation plan keeps hitting."""
        for k, v in list(self.__dict__.items()):
            if isinstance(v, torch.Tensor):
                setattr(self, k, v.to(device))
        return self

    def __repr__(self) -> str:
        e = None if self.edge_index is None else tuple(self.edge_index.shape)
        return f"Data(edge_index={e}, num_nodes={self.num_nodes})"


def download_and_extract_dataset() -> None:
    raise FileNotFoundError(
        f"MovieLens-25M is not present and this build does not download it ({MOVIELENS_25M_URL}); "
        f"place ratings.csv and movies.csv under {DATA_DIR} (or use lgcn_amd.synth for synthetic graphs)")


def to_undirected(edge_index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    """Both directions, coalesced: sorted by row * N + col, duplicates removed (PyG semantics).
    On a ROCm device: the HIP coalesce (lgcn_amd.ingest); CPU tensors keep the host path."""
    if edge_index.is_cuda:
        from lgcn_amd.ingest import to_undirected as to_undirected_hip

        return to_undirected_hip(edge_index, num_nodes)
    row, col = edge_index[0], edge_index[1]
    key = torch.cat([row * num_nodes + col, col * num_nodes + row])
    key = torch.unique(key, sorted=True)
    return torch.stack([key // num_nodes, key % num_nodes])


def _stack_union(parts: List[torch.Tensor]) -> torch.Tensor:
    return parts[0] if len(parts) == 1 else torch.cat(parts, dim=1)


class ClusterBatches(torch.utils.data.Dataset):
    """The list of per-part Data objects (train_l in the reference, :276-282)."""

    def __init__(self, items: List[Data]):
        self.items = items

    def __len__(self):
        return len(self.items)

    def __getitem__(self, i):
        return self.items[i]


def collate_union(batch: List[Data]) -> Data:
    """batch_size = 1 returns the part itself (the reference); q > 1 parts become one Data whose
    edge list is the union of theirs, global ids kept (not PyG's per-graph id offsets)."""
    if len(batch) == 1:
        return batch[0]
    return Data(edge_index=_stack_union([b.edge_index for b in batch]), num_nodes=batch[0].num_nodes,
                n_id=batch[0].n_id if hasattr(batch[0], "n_id") else None)


class MovieLensDataHandler:
    """Load MovieLens ratings, build the bipartite graph, split it and batch it for Cluster-GCN."""

    def __init__(self, ratings_path: str, movies_path: str, device: Optional[torch.device] = None,
                 min_rating: float = 4.0):
        self.ratings_path = ratings_path
        self.movies_path = movies_path
        self.device = device if device is not None else torch.device("cuda" if torch.cuda.is_available() else "cpu")
        if not os.path.exists(ratings_path) or not os.path.exists(movies_path):
            download_and_extract_dataset()
        ratings = pd.read_csv(ratings_path, usecols=["userId", "movieId", "rating"])
        ratings = ratings[ratings["rating"] >= min_rating]
        self.movies = pd.read_csv(movies_path, usecols=["movieId", "title"])
        # ids in order of first appearance == enumerate(series.unique()) of the reference
        user_codes, user_ids = pd.factorize(ratings["userId"], sort=False)
        movie_codes, movie_ids = pd.factorize(ratings["movieId"], sort=False)
        self.num_users = len(user_ids)
        self.num_movies = len(movie_ids)
        self.user_id_map: Dict[int, int] = {int(u): i for i, u in enumerate(user_ids)}
        self.id_user_map = {i: u for u, i in self.user_id_map.items()}
        self.movie_id_map: Dict[int, int] = {int(m): i + self.num_users for i, m in enumerate(movie_ids)}
        self.id_movie_map = {i: m for m, i in self.movie_id_map.items()}
        self._preprocess(np.asarray(user_codes, np.int64), np.asarray(movie_codes, np.int64) + self.num_users)

    def _preprocess(self, user_idx: np.ndarray, movie_idx: np.ndarray) -> None:
        edge_index = torch.from_numpy(np.vstack((user_idx, movie_idx))).long()
        if self.device.type == "cuda":  # coalesce on the device (HIP radix sort), keep the result on the host
            edge_index = to_undirected(edge_index.to(self.device), self.num_users + self.num_movies).cpu()
        else:
            edge_index = to_undirected(edge_index, self.num_users + self.num_movies)
        self.edge_index = edge_index

    @property
    def num_nodes(self) -> int:
        return self.num_users + self.num_movies

    def get_datasets(self, train_size: float = 0.9, indexes_path: str = "data/indexes",
                     random_state: Optional[int] = None) -> Tuple[Data, Data, Data]:
        from sklearn.model_selection import train_test_split

        val_file, test_file = "val_indices.npy", "test_indices.npy"
        num_interactions = self.edge_index.shape[1]
        if not os.path.exists(indexes_path):
            all_indices = np.arange(num_interactions)
            rs2 = None if random_state is None else random_state + 1
            train_idx, val_test = train_test_split(all_indices, train_size=train_size, shuffle=True,
                                                   random_state=random_state)
            val_idx, test_idx = train_test_split(val_test, test_size=0.5, shuffle=True, random_state=rs2)
            train_idx.sort()
            val_idx.sort()
            test_idx.sort()
            self._save_indices(val_idx, test_idx, indexes_path, val_file, test_file)
        else:
            train_idx, val_idx, test_idx = self._load_from_indices(indexes_path, num_interactions, val_file, test_file)
        N = self.num_nodes

        def make(idx):
            d = Data(edge_index=self.edge_index[:, torch.from_numpy(np.asarray(idx))].contiguous(), num_nodes=N)
            d = d.to(self.device)
            d.n_id = torch.arange(N, device=self.device)
            return d

        return make(train_idx), make(val_idx), make(test_idx)

    def _load_from_indices(self, indexes_path, num_interactions, val_index_file, test_index_file):
        if not os.path.exists(indexes_path):
            raise FileNotFoundError("Indexes path not found. Please preprocess the data first.")
        val_idx = np.sort(np.load(os.path.join(indexes_path, val_index_file)))
        test_idx = np.sort(np.load(os.path.join(indexes_path, test_index_file)))
        train_idx = np.setdiff1d(np.arange(num_interactions), np.concatenate((val_idx, test_idx)))
        assert np.all(np.diff(train_idx) > 0)
        assert np.all(np.diff(val_idx) > 0)
        assert np.all(np.diff(test_idx) > 0)
        return train_idx, val_idx, test_idx

    def _save_indices(self, val_indices, test_indices, indexes_path, val_index_file, test_index_file) -> None:
        os.makedirs(indexes_path, exist_ok=True)
        np.save(os.path.join(indexes_path, val_index_file), val_indices)
        np.save(os.path.join(indexes_path, test_index_file), test_indices)

    def get_data_training(self, num_train_clusters: int = 100, clusters_per_batch: int = 1,
                          shuffle: bool = True, partition_passes: int = 4, **split_kw):
        """(train loader over Cluster-GCN parts, val Data, test Data) (reference :256-288)."""
        train, val, test = self.get_datasets(**split_kw)
        loader, self.partition = build_cluster_loader(train.edge_index, self.num_nodes, num_train_clusters,
                                                      clusters_per_batch, shuffle, partition_passes, self.device)
        return loader, val, test

    def get_num_users_items(self) -> Tuple[int, int]:
        return len(self.user_id_map), len(self.movie_id_map)


def build_cluster_loader(train_edge_index: torch.Tensor, num_nodes: int, num_parts: int,
                         clusters_per_batch: int = 1, shuffle: bool = True, passes: int = 4,
                         device=None, part: Optional[np.ndarray] = None):
    """Partition the train graph and return (DataLoader over parts, part array)."""
    if part is None:
        part = _cluster.partition_nodes(train_edge_index, num_nodes, num_parts, passes)
    device = device if device is not None else train_edge_index.device
    items = []
    for ei in _cluster.intra_part_edges(train_edge_index, part, num_parts):
        d = Data(edge_index=torch.from_numpy(ei).to(device), num_nodes=num_nodes)
        d.n_id = torch.arange(num_nodes, device=device)
        items.append(d)
    loader = torch.utils.data.DataLoader(ClusterBatches(items), batch_size=clusters_per_batch, shuffle=shuffle,
                                         collate_fn=collate_union)
    return loader, part


def write_synthetic_movielens(directory: str, num_users: int, num_items: int, num_ratings: int,
                              seed: int = 0) -> Tuple[str, str]:
    """A ratings.csv / movies.csv pair in the MovieLens schema (userId, movieId, rating,
    timestamp / movieId, title, genres), seeded, ~half the ratings >= 4 — the build's stand-in for
    the reference's data/reviews.csv subsample (BASELINE config 0)."""
    from lgcn_amd import synth

    rng = np.random.default_rng(seed)
    u, i = synth.random_pairs(num_users, num_items, num_ratings, seed)
    user_ids = rng.permutation(np.arange(1, 10 * num_users))[:num_users]
    movie_ids = rng.permutation(np.arange(1, 10 * num_items))[:num_items]
    order = rng.permutation(u.size)
    ratings = rng.choice(np.arange(1, 11) / 2.0, size=u.size, p=[.02, .03, .03, .07, .06, .19, .13, .26, .08, .13])
    os.makedirs(directory, exist_ok=True)
    rp = os.path.join(directory, "ratings.csv")
    mp = os.path.join(directory, "movies.csv")
    pd.DataFrame({"userId": user_ids[u[order]], "movieId": movie_ids[i[order]], "rating": ratings,
                  "timestamp": 1_000_000_000 + rng.integers(0, 10 ** 8, u.size)}).to_csv(rp, index=False)
    pd.DataFrame({"movieId": movie_ids, "title": [f"Movie {m}" for m in movie_ids],
                  "genres": "Drama"}).to_csv(mp, index=False)
    return rp, mp
