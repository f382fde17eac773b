"""Row-sharded propagation (lgcn_amd.sharded), host logic on CPU, world_size 2, 3, 4 and 8 on gloo.

The HIP kernels need a GPU, so each rank's "kernel" here is a CPU stand-in (CpuShardPlan) that
computes a layer with the oracle restatement (oracle/lgconv_ref.py) and keeps only the rows the
rank owns in the half it is asked for. What is under test is the product's host side:
ownership ranges, the padded id layout, the half order of each layer, the ping-pong buffers,
the epilogue modes and the block all_gather (BlockExchange over gloo). The sharded output must be
BITWISE the one-rank oracle forward (tests/test_gpu_sharded.py runs the same with the kernels).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from lgcn_amd import _ffi
from lgcn_amd.sharded import BlockExchange, Half, RowShards, balanced_bounds, propagate_forward_sharded


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _graph(kind):
    import graphs

    if kind == "sym":
        return graphs.sym(seed=4)
    if kind == "sub":
        return graphs.subsampled(seed=5)
    if kind == "hub":
        return graphs.hub()
    # not bipartite: add user-user and item-item edges (one piece per layer, both blocks exchanged)
    U, I, ei = graphs.sym(U=80, I=60, pairs=700, seed=6)
    rng = np.random.default_rng(6)
    extra = np.stack([rng.integers(0, U + I, 300), rng.integers(0, U + I, 300)])
    key = np.unique(np.concatenate([ei[0] * (U + I) + ei[1], extra[0] * (U + I) + extra[1]]))
    return U, I, np.stack([key // (U + I), key % (U + I)])


class CpuShardPlan:
    """Stand-in for ShardedPlan on CPU: the same halves and blocks, the layer computed by the
    oracle over the padded edge list (a strictly increasing relabelling, so each row is the same
    sequential sum), the epilogue applied to the rank's rows of the half only."""

    def __init__(self, ei, shards, rank):
        from oracle import lgconv_ref as R

        self.R = R
        self.shards = shards
        self.NP = shards.NP
        pm = shards.padmap()
        self.eip = pm[ei]
        self.w = R.gcn_norm(self.eip, self.NP)
        U = shards.U
        self.bipartite = bool(np.all((ei[0] < U) != (ei[1] < U)))
        pieces = [("u", "i"), ("i", "u")] if self.bipartite else [("ui", "ui")]
        self.halves = [Half(None, r, w) for r, w in pieces]
        self.rows = [np.flatnonzero(shards.owned_mask(rank, w)) for _, w in pieces]
        self.sliced = False
        self.log = []

    def run_half(self, h, x, e, acc, y, mode, div, mul):
        rows = self.rows[self.halves.index(h)]
        self.log.append((h.reads, h.writes))
        v = torch.from_numpy(self.R.lgconv(x.numpy(), self.eip, self.w))[rows]
        if mode == _ffi.EPI_INIT:
            acc[rows] = e[rows] + v
        elif mode == _ffi.EPI_ADD:
            acc[rows] = acc[rows] + v
        elif mode == _ffi.EPI_FINAL_ACC:
            acc[rows] = ((acc[rows] + v) / div) * mul
        elif mode == _ffi.EPI_FINAL_E:
            acc[rows] = ((e[rows] + v) / div) * mul
        if y is not None and mode in (_ffi.EPI_INIT, _ffi.EPI_ADD):
            y[rows] = v


def _worker(rank, world, port, kind, K, out_dir, F=1, mode="allgather"):
    import sys

    from conftest import PKG, ROOT
    sys.path[:0] = [str(PKG), str(ROOT), str(ROOT / "tests")]
    import graphs
    from lgcn_amd.sharded import ShardGrid

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    U, I, ei = _graph(kind)
    grid = ShardGrid.build(world, rank, 16, world // F, F)
    c0, c1 = grid.cols
    g_r = grid.row_group
    deg = np.bincount(ei[1], minlength=U + I)
    shards = RowShards.build(deg, U, grid.R)
    plan = CpuShardPlan(ei, shards, g_r)
    uw, iw = graphs.embeddings(U, I, 16, seed=K)
    x0p = shards.to_padded(torch.from_numpy(uw[:, c0:c1].copy()), torch.from_numpy(iw[:, c0:c1].copy()))
    group = grid.exchange_group(dist)
    ex = BlockExchange(shards, g_r, group, grid.members, mode) if grid.R > 1 else None
    out = propagate_forward_sharded(x0p, plan, K, ex)
    a, b = shards.user_rows(g_r)
    c, d = shards.item_rows(g_r)
    np.save(os.path.join(out_dir, f"u{g_r}_{grid.col_group}.npy"), out[a:b].numpy())
    np.save(os.path.join(out_dir, f"i{g_r}_{grid.col_group}.npy"), out[c:d].numpy())
    np.save(os.path.join(out_dir, f"log{rank}.npy"), np.array(["".join(x) for x in plan.log]))
    dist.destroy_process_group()


@pytest.mark.parametrize("kind,world,K,F,mode", [("sym", 2, 3, 1, "allgather"), ("sub", 2, 3, 1, "allgather"),
                                                 ("hub", 2, 4, 1, "allgather"), ("sym", 3, 2, 1, "allgather"),
                                                 ("nonbip", 2, 3, 1, "allgather"), ("sub", 2, 1, 1, "allgather"),
                                                 ("sub", 2, 3, 2, "allgather"), ("hub", 4, 3, 2, "allgather"),
                                                 ("nonbip", 4, 2, 2, "allgather"), ("sym", 3, 2, 1, "p2p"),
                                                 ("hub", 4, 3, 2, "p2p"), ("sub", 4, 3, 1, "p2p"),
                                                 ("hub", 8, 3, 1, "p2p")])
def test_sharded_equals_single_rank_bitwise(tmp_path, kind, world, K, F, mode):
    """R = world / F row groups x F column groups (F = 2: each rank propagates 8 of the 16
    columns; ranks of one column group exchange rows, column groups exchange nothing); the rows
    travel as one all_gather per block, or as sends to / receives from every peer (p2p)."""
    from oracle import c_oracle

    port = _free_port()
    mp.spawn(_worker, args=(world, port, kind, K, str(tmp_path), F, mode), nprocs=world, join=True)
    import graphs

    U, I, ei = _graph(kind)
    uw, iw = graphs.embeddings(U, I, 16, seed=K)
    ru, ri = c_oracle.lightgcn_forward(uw, iw, ei, K)
    R = world // F
    got_u = np.concatenate([np.concatenate([np.load(tmp_path / f"u{r}_{c}.npy") for c in range(F)], axis=1)
                            for r in range(R)])
    got_i = np.concatenate([np.concatenate([np.load(tmp_path / f"i{r}_{c}.npy") for c in range(F)], axis=1)
                            for r in range(R)])
    assert np.array_equal(got_u, ru) and np.array_equal(got_i, ri)
    log = list(np.load(tmp_path / "log0.npy"))
    if kind != "nonbip":
        # layer k runs A (reads users, writes items) first when k is odd, B first when k is even
        expect = [["ui", "iu"] if k % 2 else ["iu", "ui"] for k in range(1, K + 1)]
        assert log == [x for pair in expect for x in pair]
    else:
        assert log == ["uiui"] * K


def test_row_shards_layout():
    U, I, ei = _graph("hub")
    deg = np.bincount(ei[1], minlength=U + I)
    for W in (1, 2, 3, 8):
        s = RowShards.build(deg, U, W)
        pm = s.padmap()
        assert np.all(np.diff(pm) > 0)                           # strictly increasing
        assert pm[U - 1] < s.side <= pm[U]                         # users, then items
        owned = sum(s.owned_mask(r) for r in range(W))
        assert owned.max() == 1 and owned.sum() == U + I           # every row owned exactly once
        assert set(np.flatnonzero(owned)) == set(pm.tolist())
        # edge-balanced: no rank's users carry much more than its share of the user in-edges
        eu = [deg[s.ub[r]:s.ub[r + 1]].sum() for r in range(W)]
        assert max(eu) <= deg[:U].sum() / W + deg[:U].max() + 4 * U / W
        x = torch.randn(U + I, 8)
        assert torch.equal(s.from_padded(s.to_padded(x[:U], x[U:])), x)
        # slice bounds keep every source in its slice
        bounds = [0, U // 2, U, U + I // 2, U + I]
        pb = s.pad_bounds(bounds)
        src = np.arange(U + I)
        assert np.array_equal(np.searchsorted(bounds, src, side="right"), np.searchsorted(pb, pm[src], side="right"))


def test_balanced_bounds():
    w = np.array([1, 1, 1, 100, 1, 1, 1, 1])
    b = balanced_bounds(w, 2)
    assert b[0] == 0 and b[-1] == 8 and np.all(np.diff(b) >= 0)
    assert list(balanced_bounds(np.ones(10), 5)) == [0, 2, 4, 6, 8, 10]
    b = balanced_bounds(np.ones(2), 4)  # more ranks than rows: some ranges are empty
    assert b[0] == 0 and b[-1] == 2 and len(b) == 5 and np.all(np.diff(b) >= 0)


def test_grid_shape():
    from lgcn_amd.sharded import ShardGrid, grid_shape

    assert grid_shape(1, 64) == (1, 1)
    assert grid_shape(2, 64) == (1, 2) and grid_shape(4, 64) == (2, 2) and grid_shape(8, 64) == (4, 2)
    assert grid_shape(3, 64) == (3, 1)                       # odd world: rows only
    assert grid_shape(8, 32) == (8, 1)                       # 16 columns would not cut gather requests
    assert grid_shape(8, 256) == (4, 2)
    g = ShardGrid.build(8, 5, 64)
    assert (g.R, g.F, g.row_group, g.col_group, g.cols) == (4, 2, 2, 1, (32, 64))
    with pytest.raises(ValueError):
        ShardGrid.build(8, 0, 64, 3, 2)


def test_grid_candidates():
    from lgcn_amd.sharded import grid_candidates

    assert grid_candidates(1, 64) == [(1, 1, None)]
    assert grid_candidates(2, 64) == [(1, 2, None)]
    # world >= 4: R - 1 >= 3 links; "reduce" (users sharded, items all-reduced) for every R > 1
    # peer sends (p2p) are timed after every other candidate (a hang there cannot stop the others)
    red = lambda R, F: [(R, F, "reduce"), (R, F, "reduce-fused"), (R, F, "reduce-a2a"),  # noqa: E731
                        (R, F, "reduce-a2a-fused")]
    rows_only = lambda w: [(w, 1, "allgather")] + red(w, 1)  # noqa: E731
    assert grid_candidates(4, 64) == [(1, 4, None), (2, 2, "allgather")] + red(2, 2) + rows_only(4) + \
        [(4, 1, "p2p")]
    assert grid_candidates(8, 64) == [(1, 8, None), (2, 4, "allgather")] + red(2, 4) + [(4, 2, "allgather")] + \
        red(4, 2) + rows_only(8) + [(4, 2, "p2p"), (8, 1, "p2p")]
    assert grid_candidates(3, 64) == rows_only(3) + [(3, 1, "p2p")]   # odd world: rows only
    assert grid_candidates(8, 32) == [(2, 4, "allgather")] + red(2, 4) + [(4, 2, "allgather")] + red(4, 2) + \
        rows_only(8) + [(4, 2, "p2p"), (8, 1, "p2p")]  # 4-col shares: no 1 x 8
    assert (4, 1, "reduce") not in grid_candidates(4, 64, bipartite=False)
    for R, F, _ in grid_candidates(8, 256):
        assert R * F == 8 and (256 // F) % 4 == 0


class CpuReducePlan:
    """Stand-in for ReducePlan on CPU: the three passes computed by the oracle restatement (the
    whole graph's gcn_norm weights; the item partials over the edges this row group's users source,
    summed in edge order), the epilogue applied to the rows each pass writes."""

    def __init__(self, ei, shards, g):
        from oracle import lgconv_ref as R

        self.R, self.shards = R, shards
        self.N, self.U = shards.N, shards.U
        self.ei = ei
        self.w = R.gcn_norm(ei, self.N)
        ua, ub = shards.users(g)
        self.own = np.arange(ua, ub)
        sel = (ei[0] >= ua) & (ei[0] < ub)
        self.ei_sub, self.w_sub = ei[:, sel], self.w[sel]
        self.log = []
        self.g = g
        I = self.N - self.U
        self.I_pad = -(-I // shards.R) * shards.R
        per = self.I_pad // shards.R
        self.share = (min(I, g * per), min(I, (g + 1) * per))

    @staticmethod
    def _epi(acc, e, rows, v, mode, div, mul):
        if mode == _ffi.EPI_INIT:
            acc[rows] = e[rows] + v
        elif mode == _ffi.EPI_ADD:
            acc[rows] = acc[rows] + v
        elif mode == _ffi.EPI_FINAL_ACC:
            acc[rows] = ((acc[rows] + v) / div) * mul
        elif mode == _ffi.EPI_FINAL_E:
            acc[rows] = ((e[rows] + v) / div) * mul
        elif mode == _ffi.EPI_STORE:
            acc[rows] = v

    def run_partial(self, x_users, part_items):
        self.log.append("partial")
        x = np.zeros((self.N, x_users.shape[1]), np.float32)
        x[:self.U] = x_users.numpy()
        part_items[:self.N - self.U] = torch.from_numpy(self.R.lgconv(x, self.ei_sub, self.w_sub)[self.U:])

    def run_users(self, x_items, e, acc, y, mode, div, mul):
        self.log.append("users")
        x = np.zeros((self.N, x_items.shape[1]), np.float32)
        x[self.U:] = x_items[:self.N - self.U].numpy()
        v = torch.from_numpy(self.R.lgconv(x, self.ei, self.w)[self.own])
        self._epi(acc[0], e[0] if e is not None else None, self.own, v, mode, div, mul)
        if y is not None and mode in (_ffi.EPI_INIT, _ffi.EPI_ADD):
            y[self.own] = v

    def run_pair(self, x_users, part_items, x_items, e, acc, y, mode, div, mul):
        self.run_partial(x_users, part_items)
        self.run_users(x_items, e, acc, y, mode, div, mul)

    def finish_items(self, x0i, layers, last_share, out_i, div, mul):
        self.log.append("items")
        a, b = self.share
        s = x0i[a:b].clone()
        for t in list(layers) + [last_share]:
            s = s + (t[a:b] if t is not last_share else t[:b - a])
        out_i[a:b] = (s / div) * mul


def _reduce_worker(rank, world, port, kind, K, out_dir, F=1, fused=False, method="ring"):
    import sys

    from conftest import PKG, ROOT
    sys.path[:0] = [str(PKG), str(ROOT), str(ROOT / "tests")]
    import graphs
    from lgcn_amd.sharded import ItemReducer, ShardGrid, UserShards, propagate_forward_reduced

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    U, I, ei = _graph(kind)
    grid = ShardGrid.build(world, rank, 16, world // F, F)
    c0, c1 = grid.cols
    g = grid.row_group
    shards = UserShards.build(np.bincount(ei[1], minlength=U + I), U, grid.R)
    plan = CpuReducePlan(ei, shards, g)
    uw, iw = graphs.embeddings(U, I, 16, seed=K)
    group = grid.exchange_group(dist)
    red = ItemReducer(grid.R, group, method=method)
    ou, oi = propagate_forward_reduced(torch.from_numpy(uw[:, c0:c1].copy()), torch.from_numpy(iw[:, c0:c1].copy()),
                                       plan, K, red, fused=fused)
    ua, ub = shards.users(g)
    a, b = plan.share
    np.save(os.path.join(out_dir, f"u{g}_{grid.col_group}.npy"), ou[ua:ub].numpy())
    np.save(os.path.join(out_dir, f"i{g}_{grid.col_group}.npy"), oi[a:b].numpy())
    np.save(os.path.join(out_dir, f"log{rank}.npy"), np.array(plan.log))
    dist.destroy_process_group()


@pytest.mark.parametrize("kind,world,K,F,fused,method", [
    ("sym", 2, 3, 1, False, "ring"), ("sub", 2, 3, 1, False, "ring"), ("hub", 3, 4, 1, False, "ring"),
    ("sym", 4, 2, 2, False, "ring"), ("sub", 4, 1, 1, False, "ring"), ("hub", 2, 3, 1, False, "ring"),
    ("sub", 8, 3, 2, False, "ring"), ("sym", 2, 0, 1, False, "ring"), ("hub", 3, 4, 1, True, "ring"),
    ("sub", 4, 1, 1, True, "ring"), ("sub", 8, 3, 2, True, "ring"),
    ("sub", 2, 3, 1, False, "a2a"), ("hub", 3, 4, 1, False, "a2a"), ("sub", 8, 3, 2, False, "a2a"),
    ("sub", 4, 1, 1, True, "a2a"), ("sym", 4, 2, 2, True, "a2a")])
def test_reduce_mode_matches_oracle(tmp_path, kind, world, K, F, fused, method):
    """The reduce mode (users sharded, item rows all-reduced per layer, the last layer
    reduce-scattered) over gloo: every row group's users and its share of the items within 1e-5
    per row of the one-rank oracle forward (an item row is the sum of R partial chains), the
    shares covering every item, and the pass order (the item rows' stack mean once, at the end);
    fused: the layer's two passes issued as one pair; a2a: the all_reduce as all_to_all + slice
    sums in rank order + all_gather (ItemReducer method "a2a")."""
    import graphs
    from oracle import lgconv_ref as R
    from parity import assert_rows_close

    from lgcn_amd.sharded import UserShards

    U, I, ei = _graph(kind)
    port = _free_port()
    mp.spawn(_reduce_worker, args=(world, port, kind, K, str(tmp_path), F, fused, method), nprocs=world, join=True)
    uw, iw = graphs.embeddings(U, I, 16, seed=K)
    ref = R.lightgcn_forward(uw, iw, ei, K)
    ref = np.concatenate(ref) if isinstance(ref, tuple) else ref
    shards = UserShards.build(np.bincount(ei[1], minlength=U + I), U, world // F)
    w = 16 // F
    for g in range(world // F):
        ua, ub = shards.users(g)
        got = np.concatenate([np.load(tmp_path / f"u{g}_{c}.npy") for c in range(F)], axis=1)
        assert_rows_close(got, ref[ua:ub], what=f"users of row group {g}")
    got_i = np.concatenate([np.concatenate([np.load(tmp_path / f"i{g}_{c}.npy") for c in range(F)], axis=1)
                            for g in range(world // F)])
    assert got_i.shape[0] == I  # the shares cover every item once
    assert_rows_close(got_i, ref[U:], what="items (the row groups' shares)")
    if K:
        log = list(np.load(tmp_path / "log0.npy"))
        expect = ["partial", "users"] * K + ["items"]
        assert log == expect, log


def test_grid_candidates_without_p2p():
    from lgcn_amd.sharded import grid_candidates

    for world in (3, 4, 8):
        full = grid_candidates(world, 64)
        assert grid_candidates(world, 64, p2p=False) == [c for c in full if c[2] != "p2p"]
        assert any(c[2] == "p2p" for c in full)
