"""The C1-size training + Recall harness shared by tests/test_noise_floor.py (CPU) and
tests/test_gpu_training.py::test_recall_parity_c1_size (GPU).

BASELINE configs[0]'s size: U = 1000, I = 600, 25k pairs -> E = 50k directed edges, K = 2, d = 64;
a 90 / 5 / 5 split, 4 Cluster-GCN parts, one part per step (the reference's batch_size = 1,
data/dataset_handler.py:285), 5 epochs of the reference harness (utils/train_test.py train:
Adam 1e-3, clip_grad_norm_(1)), then Recall@20 / @100 on the 2,500 validation edges
(compute_embeddings + compute_recall_at_k, numpy seed 5). Negatives come from one CPU generator
(seed 31) whatever the device, so every run trains on the same triplets.

order_seed (oracle only): a second valid summation order — each layer's edges and each batch's
triplets permuted (the same triplets, the same sums in another order) — the oracle's own noise
floor."""
from __future__ import annotations

import contextlib

import numpy as np
import torch

EPOCHS, PARTS = 5, 4


class _Batch:
    def __init__(self, ei):
        self.edge_index = ei

    def to(self, device):
        return _Batch(self.edge_index.to(device))


def c1_data():
    from lgcn_amd import cluster, synth

    g = synth.bipartite(1000, 600, 25_000, seed=11)
    U, I, E = g.num_users, g.num_items, g.num_edges
    perm = np.random.default_rng(0).permutation(E)
    n_tr, n_va = int(0.9 * E), int(0.05 * E)
    train = np.ascontiguousarray(g.edge_index[:, np.sort(perm[:n_tr])])
    val = np.ascontiguousarray(g.edge_index[:, np.sort(perm[n_tr:n_tr + n_va])])
    _, _, parts = cluster.cluster_batches(train, U + I, PARTS, 1)
    return U, I, [p for p in parts if p.shape[1]], val


@contextlib.contextmanager
def cpu_negatives(seed: int):
    """utils.helpers.sample_negative drawing from one CPU generator, then moved to the device."""
    from utils import helpers

    gen = torch.Generator().manual_seed(seed)
    orig = helpers.sample_negative

    def sample_negative(pos_idx, num_items, device):
        return torch.randint(0, num_items, (pos_idx.shape[0],), generator=gen).to(device)

    helpers.sample_negative = sample_negative
    try:
        yield gen
    finally:
        helpers.sample_negative = orig


@contextlib.contextmanager
def second_order(model, seed: int):
    """A second valid summation order for the oracle model's harness: every LGConv call sums its
    edges in a permuted order, every batch's triplets are taken in a permuted order."""
    from oracle.lgconv_torch import lgconv_torch
    from utils import helpers
    from utils import train_test as TT

    rng = torch.Generator().manual_seed(seed)

    def conv(x, ei):
        return lgconv_torch(x, ei[:, torch.randperm(ei.shape[1], generator=rng)])

    for c in model.convs:
        c.forward = conv
    orig = TT.get_triplets_indices

    def trip(ei, nu, ni, dev):
        u, p, n = helpers.get_triplets_indices(ei, nu, ni, dev)
        q = torch.randperm(u.numel(), generator=rng)
        return u[q], p[q], n[q]

    TT.get_triplets_indices = trip
    try:
        yield
    finally:
        TT.get_triplets_indices = orig


def init_state():
    from oracle.lgconv_torch import OracleLightGCN

    U, I, _, _ = c1_data()
    torch.manual_seed(0)
    return OracleLightGCN(U, I, num_layers=2, dim_h=64).state_dict()


def train_c1(device, order_seed: int | None = None, data=None, init=None):
    """(model, gen state after training): 5 epochs of the reference harness on the oracle model
    (device cpu) or this package's LightGCN (a ROCm device)."""
    from models.light_gcn import LightGCN
    from oracle.lgconv_torch import OracleLightGCN
    from utils import train_test as TT

    U, I, parts, _ = data or c1_data()
    init = init if init is not None else init_state()
    if device.type == "cpu":
        m = OracleLightGCN(U, I, num_layers=2, dim_h=64)
    else:
        m = LightGCN(U, I, num_layers=2, dim_h=64).to(device)
    m.load_state_dict(init)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    with cpu_negatives(31) as gen, (second_order(m, order_seed) if order_seed is not None else contextlib.nullcontext()):
        for _ in range(EPOCHS):
            TT.train(m, opt, [_Batch(torch.from_numpy(p)) for p in parts], device)
        path = TT.LAST_TRAIN_PATH
        state = gen.get_state()
    return m, state, path


def tables(m):
    return m.user_embedding.weight.detach().cpu().clone(), m.item_embedding.weight.detach().cpu().clone()


def recall(w, device, gen_state, data=None, ks=(20, 100)):
    """Recall@k of tables w = (user, item) on the validation edges, scored on `device` (the CPU
    reference formula on a CPU; lgcn_amd.recall on a ROCm device, under the current tuning's
    recall_ties), the validation negatives drawn from the generator state the training left."""
    from models.light_gcn import LightGCN
    from oracle.lgconv_torch import OracleLightGCN
    from utils import train_test as TT

    U, I, _, val = data or c1_data()
    m = OracleLightGCN(U, I, num_layers=2, dim_h=64) if device.type == "cpu" else \
        LightGCN(U, I, num_layers=2, dim_h=64).to(device)
    with torch.no_grad():
        m.user_embedding.weight.copy_(w[0])
        m.item_embedding.weight.copy_(w[1])
    with cpu_negatives(0) as gen:
        gen.set_state(gen_state)
        with torch.no_grad():
            embs = TT.compute_embeddings(m, _Batch(torch.from_numpy(val)).to(device), device)
            out = {}
            for k in ks:
                np.random.seed(5)
                out[k] = TT.compute_recall_at_k((embs[1], embs[3], embs[5]), k=k)
    return out
