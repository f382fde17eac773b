"""Data-parallel Cluster-GCN training over torch.distributed, world_size 2 on gloo (CPU).

The HIP propagation needs a GPU, so the model here is the CPU oracle LightGCN; what is under
test is the distributed logic the product path shares (lgcn_amd.distributed): batch sharding,
gradient all-reduce, identical optimizer steps on every rank, global loss reduction."""
import os
import socket
import types

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from lgcn_amd import distributed as D


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Batch:
    def __init__(self, ei):
        self.edge_index = ei

    def to(self, device):
        return self


def _batches():
    from lgcn_amd import cluster, synth

    g = synth.bipartite(120, 80, 1500, seed=9)
    part = cluster.partition_nodes(g.edge_index, g.num_nodes, 6)
    return g.num_users, g.num_items, [_Batch(torch.from_numpy(x)) for x in cluster.intra_part_edges(g.edge_index, part, 6)]


def _worker(rank, world, port, out_dir):
    import sys

    from conftest import PKG, ROOT
    sys.path[:0] = [str(PKG), str(ROOT)]
    from oracle.lgconv_torch import OracleLightGCN

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    U, I, batches = _batches()
    torch.manual_seed(0)
    model = OracleLightGCN(U, I, num_layers=2, dim_h=16)
    opt = torch.optim.Adam(model.parameters(), lr=1e-2)
    losses = []
    for epoch in range(3):
        torch.manual_seed(100 + 10 * epoch + rank)  # per-rank negatives
        losses.append(D.train_epoch(model, opt, batches, torch.device("cpu"), seed=1, epoch=epoch))
    np.save(os.path.join(out_dir, f"w{rank}.npy"),
            np.concatenate([model.user_embedding.weight.detach().numpy(), model.item_embedding.weight.detach().numpy()]))
    np.save(os.path.join(out_dir, f"l{rank}.npy"), np.array(losses))
    dist.destroy_process_group()


def test_two_rank_dp_keeps_replicas_identical(tmp_path):
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    w0, w1 = np.load(tmp_path / "w0.npy"), np.load(tmp_path / "w1.npy")
    l0, l1 = np.load(tmp_path / "l0.npy"), np.load(tmp_path / "l1.npy")
    assert np.array_equal(w0, w1)           # identical replicas after every step
    assert np.array_equal(l0, l1)           # one global loss
    assert np.all(np.isfinite(l0)) and l0[-1] < l0[0]


def test_rank_share_partitions_the_epoch():
    n, world = 11, 4
    shares = [D.rank_share(n, world, r, seed=3, epoch=2) for r in range(world)]
    flat = [b for s in shares for b in s]
    assert len(flat) == (n // world) * world and len(set(flat)) == len(flat)
    assert all(len(s) == n // world for s in shares)
    with pytest.raises(ValueError):
        D.rank_share(2, 4, 0, 0, 0)


def test_single_rank_equals_reference_train():
    """W = 1: train_epoch is the reference train() over the epoch's shuffled order."""
    from oracle.lgconv_torch import OracleLightGCN
    from utils import train_test as TT

    U, I, batches = _batches()
    order = D.rank_share(len(batches), 1, 0, seed=5, epoch=0)
    res = []
    for fn in ("dp", "ref"):
        torch.manual_seed(0)
        m = OracleLightGCN(U, I, num_layers=2, dim_h=16)
        opt = torch.optim.Adam(m.parameters(), lr=1e-2)
        torch.manual_seed(77)
        if fn == "dp":
            loss = D.train_epoch(m, opt, batches, torch.device("cpu"), seed=5, epoch=0)
        else:
            loss = TT.train(m, opt, [batches[b] for b in order], torch.device("cpu"))
        res.append((loss, m.user_embedding.weight.detach().clone()))
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1], res[1][1])


def _hybrid_worker(rank, world, port, out_dir):
    import sys

    from conftest import PKG, ROOT
    sys.path[:0] = [str(PKG), str(ROOT)]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    U, I, batches = _batches()
    cap = D.user_exchange_capacity(batches, U)
    gi = torch.full((I, 4), float(rank + 1))  # rank r's item gradient table: r + 1 everywhere
    ex = D.HybridExchange(cap, U, gi, torch.device("cpu"), world)
    ex.ids.fill_(-1)
    ex.ids[:2] = torch.tensor([rank, U - 1 - rank])  # two user records per rank
    ex.rows[:2] = float(10 * (rank + 1))
    ex.gather()
    np.save(os.path.join(out_dir, f"h{rank}.npy"), np.concatenate([
        np.array([cap, ex.bytes], dtype=np.float64), gi.numpy().ravel().astype(np.float64),
        ex.pack_all.view(world, ex.blk)[:, :2 * ex.cap].contiguous().view(torch.int64)[:, :2].numpy().ravel()
        .astype(np.float64)]))
    dist.destroy_process_group()


def test_two_rank_hybrid_exchange_gathers_users_and_sums_items(tmp_path):
    """HybridExchange (lgcn_amd.distributed) over gloo, world 2: the users' record blocks are
    all-gathered in rank order, the item gradient table is summed in place on every rank, and the
    capacity is the most user rows any batch touches."""
    port = _free_port()
    mp.spawn(_hybrid_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    U, I, batches = _batches()
    want_cap = max(int((torch.unique(b.edge_index) < U).sum()) for b in batches)
    h0, h1 = np.load(tmp_path / "h0.npy"), np.load(tmp_path / "h1.npy")
    assert np.array_equal(h0, h1)  # every rank: the same capacity, bytes, sums and gathered ids
    assert int(h0[0]) == want_cap
    items = h0[2:2 + I * 4]
    assert np.all(items == 3.0)  # 1 + 2 on both ranks
    ids = h0[2 + I * 4:].reshape(2, 2)
    assert ids.tolist() == [[0, U - 1], [1, U - 2]]  # rank order


def test_exchange_capacity_holds_dense_batches():
    """VERDICT r5 weak #9 (gpurun_out/r05zk/c4proj_planted.log: 'lgcn_rows_pack: bad args
    (n_a=6869 n_b=178333 cap=65968)'). lgcn_rows_pack is position-based — a slot per touched row
    plus one per triplet's negative, first occurrence or not — so a rank's record block needs
    touched + B slots. The failing projection ran an uncommitted sizing by DISTINCT rows (65,968 =
    6,921 touched + I = 59,047 items, the owner exchange's dedupe rule applied to the replicated
    block); the committed exchange_capacity counts touched + B. Pinned here on a planted graph whose
    batches draw more negatives than there are items (B > I, as the planted C3 batches do)."""
    from lgcn_amd import cluster, synth

    g, _ = synth.planted_ml25m(64, scale=0.02)
    U, I = g.num_users, g.num_items
    _, _, lists = cluster.cluster_batches(g.edge_index, g.num_nodes, 64, 8)
    batches = [types.SimpleNamespace(edge_index=torch.from_numpy(x)) for x in lists if x.shape[1]]
    cap = D.exchange_capacity(batches, U)
    need, dense = 0, 0
    for b in batches:
        ei = b.edge_index
        touched = int(torch.unique(ei).numel())
        B = int((ei[0] < U).sum())
        need = max(need, touched + B)
        dense += B > I
        assert cap >= touched + B
    assert dense > 0, "no batch draws more negatives than there are items"
    assert cap == need
    ex = D.RowExchange(cap, U + I, 4, torch.device("cpu"), 1)
    assert ex.cap >= need and ex.cap % 2 == 0
