"""Host logic of the round-3 multi-GPU training modes, on CPU (no kernels): the owner-sharded
exchange's capacities and block layout (lgcn_amd.owner), and the column-sharded ColumnGroup's
column shares, reg coefficient and collectives (world 2 over gloo)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class _Batch:
    def __init__(self, ei):
        self.edge_index = ei


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_owner_capacity_bounded_by_the_owners_items():
    """A batch with more triplets than items (the planted graph's 180k triplets over 59k items):
    each destination carries each distinct row once (first-occurrence gradient rows, claimed
    requests), so given num_items its block needs its touched rows plus at most its ceil(I / W)
    items, not its share of B."""
    from lgcn_amd.owner import owner_capacity

    rng = np.random.default_rng(1)
    U, I = 400, 30
    u = rng.integers(0, U, 2000)
    i = rng.integers(0, I, 2000) + U
    ei = np.unique(np.stack([np.concatenate([u, i]), np.concatenate([i, u])]), axis=1)
    b = _Batch(torch.from_numpy(ei))
    assert int((ei[0] < U).sum()) > I
    t = np.unique(ei)
    for W in (2, 4, 8):
        per_owner = int(np.bincount(t % W, minlength=W).max())
        cap = owner_capacity([b], U, W, num_items=I)
        want = per_owner + -(-I // W)
        assert cap == want + want % 2
        assert cap < owner_capacity([b], U, W)


def test_owner_capacity_bounds_every_destination():
    """Per destination: the most touched rows any batch has on one owner (row r -> r % W) plus
    the negatives' expected share with slack; even (16-byte aligned rows)."""
    from lgcn_amd.owner import owner_capacity

    rng = np.random.default_rng(0)
    U, I = 300, 200
    batches = []
    for _ in range(5):
        u = rng.integers(0, U, 400)
        i = rng.integers(0, I, 400) + U
        ei = np.unique(np.stack([np.concatenate([u, i]), np.concatenate([i, u])]), axis=1)
        batches.append(_Batch(torch.from_numpy(ei)))
    for W in (1, 2, 3, 8):
        cap = owner_capacity(batches, U, W)
        assert cap % 2 == 0
        for b in batches:
            t = torch.unique(b.edge_index)
            per_owner = int(torch.bincount(t % W, minlength=W).max())
            B = int((b.edge_index[0] < U).sum())
            assert cap >= per_owner + int(np.ceil(B / W * 1.25)) + 64


def test_owner_exchange_block_layout():
    from lgcn_amd.owner import OwnerExchange

    ex = OwnerExchange(202, 1001, 64, "cpu", 1, 0, 2048)
    assert ex.req_off == 2 * 202 + 202 * 64
    assert ex.blk % 4 == 0 and ex.blk >= ex.req_off + 2 * ex.rcap
    assert ex.send.numel() == ex.blk and ex.ids_all.numel() == 202
    assert torch.equal(ex.owned, torch.arange(0, 1001))
    with pytest.raises(ValueError):
        OwnerExchange(201, 10, 64, "cpu", 1, 0, 2048)  # odd capacity: rows would lose 16-byte alignment


def test_owner_exchange_unpack_reads_the_received_blocks():
    """unpack(): the gradient ids and the request ids of every source block, -1 where empty."""
    from lgcn_amd.owner import OwnerExchange

    ex = OwnerExchange(4, 50, 8, "cpu", 1, 0, 16)
    blk = ex.recv.view(1, ex.blk)
    ids = torch.tensor([7, 3, -1, -1], dtype=torch.int64)
    req = torch.tensor([9, -1, 11, -1], dtype=torch.int64)
    blk[0, :8].copy_(ids.view(torch.float32))
    blk[0, ex.req_off:ex.req_off + 8].copy_(req.view(torch.float32))
    ex.unpack()
    assert torch.equal(ex.ids_all, ids) and torch.equal(ex.req_all, req)
    assert ex.req_valid.tolist() == [1, 0, 1, 0]


def test_column_group_shares():
    from lgcn_amd.train_step import ColumnGroup

    cg = ColumnGroup(8, 3, 64)
    assert cg.d == 8 and cg.cols == (24, 32)
    # the reg scale of the full width: c * 2 / (B * d) over the share == coeff * 2 / (B * d_full)
    B = 1000
    k_share = np.float32(cg.reg_coeff(5e-3)) * np.float32(2) / (np.float32(B) * np.float32(cg.d))
    k_full = np.float32(5e-3) * np.float32(2) / (np.float32(B) * np.float32(64))
    assert abs(float(k_share) - float(k_full)) <= 2 * np.spacing(np.float32(k_full))
    with pytest.raises(ValueError):
        ColumnGroup(3, 0, 64)  # 64 / 3 columns
    with pytest.raises(ValueError):
        ColumnGroup(32, 0, 64)  # 2 columns: not a multiple of 4


def _cols_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from lgcn_amd.train_step import ColumnGroup

    cg = ColumnGroup(world, rank, 16)
    t = torch.full((6,), float(rank + 1))
    cg.all_reduce(t)
    parts = cg.gather_partials(torch.arange(4, dtype=torch.float32) + 10 * rank)
    torch.save({"sum": t, "parts": parts}, os.path.join(out, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_column_group_collectives_world2(tmp_path):
    """The [B, 6] sums all-reduced over the column groups; the norm partials gathered in rank order."""
    mp.spawn(_cols_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        res = torch.load(tmp_path / f"r{r}.pt", weights_only=True)
        assert torch.equal(res["sum"], torch.full((6,), 3.0))
        assert res["parts"].tolist() == [0, 1, 2, 3, 10, 11, 12, 13]


def _dc_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from lgcn_amd.distributed import device_collectives

    from lgcn_amd import tuning

    plain = device_collectives()
    with tuning.tuned(device_collectives=True):
        forced = device_collectives()
    torch.save({"plain": plain, "forced": forced}, os.path.join(out, f"dc{rank}.pt"))
    dist.destroy_process_group()


def test_device_collectives_switch(tmp_path):
    """device_collectives(): False on a gloo group, True with tuning device_collectives=True (how the
    GPU tests send gloo runs down the RCCL branches)."""
    mp.spawn(_dc_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        res = torch.load(tmp_path / f"dc{r}.pt", weights_only=True)
        assert res == {"plain": False, "forced": True}
