"""Row-sharded propagation (lgcn_amd.sharded) with the HIP kernels: the sharded K-layer forward is
BITWISE the one-GPU forward (lgcn_amd.propagate_forward over PropagationPlan(side_split=U)),
every rank's rows, for the plain and the source-sliced schedules, with hub rows cut into chunks.
One row group (R = 1) with F column groups: each column share is bitwise the one-GPU forward of
that share at its own width (a rank slices the source range for its width); R > 1: bitwise the
full-width one-GPU forward on the plain schedule (its chunks do not depend on the width).

W = 1 runs in this process; W = 2 runs two ranks on the one GPU of the box over gloo (the block
all_gather goes through host memory; the 8-GPU RCCL run is bench.py --gpus N)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

# (graph, K, d, chunk, tuning slice_mb or None)
CASES = {
    "ml25m5_plain": ("ml25m", 3, 64, 256, None),
    "ml25m5_sliced": ("ml25m", 3, 64, 64, "0.7"),
    "hub_sliced": ("hub", 4, 32, 16, "0.05"),
    "sub_K2_d128": ("sub", 2, 128, 8, None),
}


def _graph(kind):
    import graphs
    from lgcn_amd import synth

    if kind == "ml25m":
        g = synth.ml25m_shaped(seed=5, scale=0.05)
        return g.num_users, g.num_items, g.edge_index
    if kind == "hub":
        return graphs.hub(U=3000, I=60)
    return graphs.subsampled(U=400, I=300, pairs=6000, seed=2)


def _reference(dev, case, R=1, F=1):
    """One-GPU forward with the schedule a rank of R row groups runs: the default one (R = 1; with
    F column groups, each column share run at its own width), or the plain schedule at
    lgcn_amd.sharded.rank_chunk (R > 1). Returns (..., out, sched, hub rows over the shares)."""
    from lgcn_amd import propagate_forward
    from lgcn_amd.plan import PropagationPlan
    from lgcn_amd.sharded import rank_chunk

    kind, K, d, chunk, slice_mb = CASES[case]
    U, I, ei = _graph(kind)
    import graphs

    uw, iw = graphs.embeddings(U, I, d, seed=K + d)
    from lgcn_amd import tuning

    Fw = F if R == 1 else 1
    w = d // Fw
    with tuning.tuned(**({"slice_mb": 0.0} if R > 1 else {})):
        plan = PropagationPlan(torch.from_numpy(ei).to(dev), U + I, rank_chunk(chunk, R), side_split=U)
        outs = [propagate_forward(torch.from_numpy(uw[:, c * w:(c + 1) * w].copy()).to(dev),
                                  torch.from_numpy(iw[:, c * w:(c + 1) * w].copy()).to(dev), plan, K).cpu().numpy()
                for c in range(Fw)]
        sched = plan.schedule("fwd", w)
    return U, I, ei, uw, iw, np.concatenate(outs, axis=1), sched, F * sched.n_splits


def _sharded(dev, case, world, rank, F=1, mode="allgather"):
    from lgcn_amd.sharded import BlockExchange, RowShards, ShardedPlan, ShardGrid, propagate_forward_sharded

    kind, K, d, chunk, slice_mb = CASES[case]
    U, I, ei = _graph(kind)
    import graphs

    uw, iw = graphs.embeddings(U, I, d, seed=K + d)
    grid = ShardGrid.build(world, rank, d, world // F, F)
    c0, c1 = grid.cols
    g_r = grid.row_group
    shards = RowShards.build(np.bincount(ei[1], minlength=U + I), U, grid.R)
    splan = ShardedPlan(torch.from_numpy(ei).to(dev), shards, g_r, c1 - c0, chunk)
    x0p = shards.to_padded(torch.from_numpy(uw[:, c0:c1].copy()).to(dev), torch.from_numpy(iw[:, c0:c1].copy()).to(dev))
    import torch.distributed as dist

    group = grid.exchange_group(dist) if world > 1 else None
    ex = BlockExchange(shards, g_r, group, grid.members, mode) if grid.R > 1 else None
    out = propagate_forward_sharded(x0p, splan, K, ex).cpu().numpy()
    a, b = shards.user_rows(g_r)
    c, e = shards.item_rows(g_r)
    return shards, splan, out[a:b], out[c:e]


@pytest.mark.parametrize("case", list(CASES))
def test_sharded_w1_bitwise(gpu, tune, case):
    slice_mb = CASES[case][4]
    if slice_mb:
        tune(slice_mb=float(slice_mb))
    U, I, ei, uw, iw, ref, sched, _ = _reference(gpu, case)
    shards, splan, ou, oi = _sharded(gpu, case, 1, 0)
    assert shards.NP == U + I and splan.sliced == hasattr(sched, "launches")
    assert splan.bipartite and len(splan.halves) == 2
    assert np.array_equal(ou, ref[:U]) and np.array_equal(oi, ref[U:])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case, out_dir, F=1, mode="allgather", dc=False):
    import sys

    from conftest import PKG, ROOT
    sys.path[:0] = [str(PKG), str(ROOT), str(ROOT / "tests")]
    import torch.distributed as dist

    from lgcn_amd import tuning

    slice_mb = CASES[case][4]
    if slice_mb:
        tuning.set_tuning(slice_mb=float(slice_mb))
    if dc:  # the RCCL branch's code (side stream, events, in-place device collectives) over gloo
        tuning.set_tuning(device_collectives=True)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    shards, splan, ou, oi = _sharded(dev, case, world, rank, F, mode)
    g_r, c_g = rank // F, rank % F
    np.save(os.path.join(out_dir, f"u{g_r}_{c_g}.npy"), ou)
    np.save(os.path.join(out_dir, f"i{g_r}_{c_g}.npy"), oi)
    np.save(os.path.join(out_dir, f"n{rank}.npy"),
            np.array([sum(getattr(h.direction, "n_splits", 0) for h in splan.halves), int(splan.sliced)]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("case,world,F,mode", [(c, 2, 1, "allgather") for c in CASES] +
                         [("ml25m5_sliced", 2, 2, "allgather"), ("hub_sliced", 2, 2, "allgather"),
                          ("ml25m5_sliced", 4, 2, "allgather"), ("sub_K2_d128", 4, 2, "allgather"),
                          ("ml25m5_plain", 3, 1, "p2p"), ("hub_sliced", 4, 2, "p2p")])
def test_sharded_ranks_bitwise(gpu, tune, tmp_path, case, world, F, mode):
    """world / F row groups x F column groups (gloo, every rank on the one GPU): the assembled
    output is bitwise the one-GPU forward with the schedule the ranks run (R = 1: each column share
    at its width; R > 1: lgcn_amd.sharded.rank_chunk at the full width); with R > 1 also within
    1e-5 per row of the default one."""
    _check_sharded_ranks(gpu, tune, tmp_path, case, world, F, mode, False)


@pytest.mark.parametrize("case,world,F,mode", [("ml25m5_sliced", 4, 2, "allgather"), ("hub_sliced", 4, 2, "p2p"),
                                               ("ml25m5_plain", 3, 1, "p2p"), ("sub_K2_d128", 2, 1, "allgather")])
def test_sharded_ranks_device_collectives(gpu, tune, tmp_path, case, world, F, mode):
    """The same, down the RCCL branch of BlockExchange (tuning device_collectives=True: in-place
    all_gather_into_tensor / batch_isend_irecv on CUDA tensors, on a side stream the compute
    stream waits on through events), with gloo carrying the bytes: bitwise the one-GPU forward."""
    _check_sharded_ranks(gpu, tune, tmp_path, case, world, F, mode, True)


def _check_sharded_ranks(gpu, tune, tmp_path, case, world, F, mode, dc):
    slice_mb = CASES[case][4]
    if slice_mb:
        tune(slice_mb=float(slice_mb))
    R = world // F
    U, I, ei, uw, iw, ref, sched, n_hubs = _reference(gpu, case, R, F)
    torch.cuda.synchronize()
    mp.spawn(_worker, args=(world, _free_port(), case, str(tmp_path), F, mode, dc), nprocs=world, join=True)
    got_u = np.concatenate([np.concatenate([np.load(tmp_path / f"u{r}_{c}.npy") for c in range(F)], axis=1)
                            for r in range(R)])
    got_i = np.concatenate([np.concatenate([np.load(tmp_path / f"i{r}_{c}.npy") for c in range(F)], axis=1)
                            for r in range(R)])
    assert np.array_equal(got_u, ref[:U]) and np.array_equal(got_i, ref[U:])
    if R > 1:
        from parity import assert_rows_close

        default = _reference(gpu, case, 1)[5]
        assert_rows_close(np.concatenate([got_u, got_i]), default, what="sharded vs default schedule")
    meta = [np.load(tmp_path / f"n{r}.npy") for r in range(world)]
    assert all(int(m[1]) == int(hasattr(sched, "launches")) for m in meta)
    # the hub rows (chunked in both) are split between the row groups, none lost
    assert sum(int(m[0]) for m in meta) == n_hubs


def _reduce_worker(rank, world, port, case, out_dir, F=1, dc=False, fused=False, method="ring"):
    import sys

    from conftest import PKG, ROOT
    sys.path[:0] = [str(PKG), str(ROOT), str(ROOT / "tests")]
    import torch.distributed as dist

    if dc:
        from lgcn_amd import tuning

        tuning.set_tuning(device_collectives=True)

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    import graphs
    from lgcn_amd.sharded import ItemReducer, ReducePlan, ShardGrid, UserShards, propagate_forward_reduced

    kind, K, d, chunk, _ = CASES[case]
    U, I, ei = _graph(kind)
    uw, iw = graphs.embeddings(U, I, d, seed=K + d)
    grid = ShardGrid.build(world, rank, d, world // F, F)
    c0, c1 = grid.cols
    shards = UserShards.build(np.bincount(ei[1], minlength=U + I), U, grid.R)
    rplan = ReducePlan(torch.from_numpy(ei).to(dev), shards, grid.row_group, c1 - c0, chunk)
    red = ItemReducer(grid.R, grid.exchange_group(dist), method=method)
    ou, oi = propagate_forward_reduced(torch.from_numpy(uw[:, c0:c1].copy()).to(dev),
                                       torch.from_numpy(iw[:, c0:c1].copy()).to(dev), rplan, K, red, fused=fused)
    ua, ub = shards.users(grid.row_group)
    a, b = rplan.share
    np.save(os.path.join(out_dir, f"u{grid.row_group}_{grid.col_group}.npy"), ou[ua:ub].cpu().numpy())
    np.save(os.path.join(out_dir, f"i{grid.row_group}_{grid.col_group}.npy"), oi[a:b].cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("case,world,F", [("ml25m5_plain", 2, 1), ("ml25m5_plain", 4, 2), ("hub_sliced", 3, 1),
                                          ("sub_K2_d128", 4, 1), ("ml25m5_sliced", 8, 2)])
def test_reduce_mode_ranks_match_oracle(gpu, tmp_path, case, world, F):
    """The reduce mode with the HIP kernels (gloo, every rank on the one GPU): users of every row
    group and every row group's share of the items (the last layer reduce-scattered) within 1e-5
    per row of the C oracle forward; the shares cover every item."""
    _check_reduce_ranks(gpu, tmp_path, case, world, F, False)


@pytest.mark.parametrize("case,world,F", [("ml25m5_plain", 4, 2), ("ml25m5_sliced", 8, 2), ("hub_sliced", 3, 1)])
def test_reduce_mode_device_collectives(gpu, tmp_path, case, world, F):
    """The same down ItemReducer's RCCL branch (tuning device_collectives=True: all_reduce and the last
    layer's reduce_scatter_tensor on CUDA tensors, side stream + events), gloo carrying the bytes."""
    _check_reduce_ranks(gpu, tmp_path, case, world, F, True)


@pytest.mark.parametrize("case,world,F", [("ml25m5_plain", 4, 2), ("ml25m5_sliced", 8, 1), ("sub_K2_d128", 2, 1)])
def test_reduce_mode_fused_pairs(gpu, tmp_path, case, world, F):
    """The fused order (a layer's partial and user passes as one lgcn_spmm_pair launch, their combines
    as another) within 1e-5 of the oracle, and bitwise the overlapped order's output."""
    fused_dir = tmp_path / "fused"
    fused_dir.mkdir()
    _check_reduce_ranks(gpu, fused_dir, case, world, F, False, fused=True)
    plain_dir = tmp_path / "plain"
    plain_dir.mkdir()
    _check_reduce_ranks(gpu, plain_dir, case, world, F, False)
    files = sorted(p.name for p in fused_dir.glob("*.npy"))
    assert files and files == sorted(p.name for p in plain_dir.glob("*.npy"))
    for f in files:
        assert np.array_equal(np.load(fused_dir / f), np.load(plain_dir / f)), f


@pytest.mark.parametrize("case,world,F,fused", [("ml25m5_plain", 4, 2, False), ("ml25m5_sliced", 8, 2, False),
                                                ("hub_sliced", 3, 1, True), ("sub_K2_d128", 2, 1, False)])
def test_reduce_mode_a2a_device_collectives_bitwise_host_path(gpu, tmp_path, case, world, F, fused):
    """ItemReducer method "a2a" (all_to_all_single of the partial tables' slices, the owner's
    slice sum in rank order by lgcn_stack_mean_rows, all_gather_into_tensor; the last layer stops
    after the sum): the RCCL branch's code (device collectives on a side stream, gloo carrying the
    bytes) within 1e-5 of the oracle and bitwise the same algorithm through host memory."""
    dev_dir, host_dir = tmp_path / "dc", tmp_path / "host"
    dev_dir.mkdir()
    host_dir.mkdir()
    _check_reduce_ranks(gpu, dev_dir, case, world, F, True, fused=fused, method="a2a")
    _check_reduce_ranks(gpu, host_dir, case, world, F, False, fused=fused, method="a2a")
    files = sorted(p.name for p in dev_dir.glob("*.npy"))
    assert files and files == sorted(p.name for p in host_dir.glob("*.npy"))
    for f in files:
        assert np.array_equal(np.load(dev_dir / f), np.load(host_dir / f)), f


def _check_reduce_ranks(gpu, tmp_path, case, world, F, dc, fused=False, method="ring"):
    import graphs
    from oracle import c_oracle
    from parity import assert_rows_close

    from lgcn_amd.sharded import UserShards

    kind, K, d, chunk, _ = CASES[case]
    U, I, ei = _graph(kind)
    uw, iw = graphs.embeddings(U, I, d, seed=K + d)
    ru, ri = c_oracle.lightgcn_forward(uw, iw, ei, K)
    torch.cuda.synchronize()
    mp.spawn(_reduce_worker, args=(world, _free_port(), case, str(tmp_path), F, dc, fused, method), nprocs=world,
             join=True)
    R = world // F
    shards = UserShards.build(np.bincount(ei[1], minlength=U + I), U, R)
    w = d // F
    for g in range(R):
        ua, ub = shards.users(g)
        got = np.concatenate([np.load(tmp_path / f"u{g}_{c}.npy") for c in range(F)], axis=1)
        assert_rows_close(got, ru[ua:ub], what=f"users of row group {g}")
    got_i = np.concatenate([np.concatenate([np.load(tmp_path / f"i{g}_{c}.npy") for c in range(F)], axis=1)
                            for g in range(R)])
    assert got_i.shape[0] == I
    assert_rows_close(got_i, ri, what="items (the row groups' shares)")
