"""Row-sparse gradient exchange for data-parallel training (csrc/lgcn_exchange.hip,
lgcn_amd.distributed.RowExchange): the kernels against a sequential restatement, the W = 1
exchange against the plain row-lazy step, and a 2-rank run (gloo, one GPU, one child process
per rank) against the dense all_reduce + FusedAdam data-parallel step."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu


class _Batch:
    def __init__(self, ei):
        self.edge_index = ei

    def to(self, device):
        return self


def _pack(lib, g, U, d, rows_a, keys_b, first_b, skip_b, cap, gpu):
    from lgcn_amd import _ffi

    ids = torch.empty(cap, dtype=torch.int64, device=gpu)
    rows = torch.empty((cap, d), dtype=torch.float32, device=gpu)
    _ffi.check(lib.lgcn_rows_pack(g[:U].data_ptr(), g[U:].data_ptr(), U, d, rows_a.data_ptr(), rows_a.numel(),
                                  keys_b.data_ptr(), keys_b.numel(), U, first_b.data_ptr(), skip_b.data_ptr(), cap,
                                  ids.data_ptr(), rows.data_ptr(), _ffi.stream_of(gpu)), "lgcn_rows_pack")
    return ids, rows


@pytest.mark.parametrize("records", [False, True])
@pytest.mark.parametrize("d", [64, 128])
def test_exchange_kernels_match_sequential_restatement(gpu, d, records):
    """pack (3 ranks' lists with duplicates, filters, padding) -> mark_first -> accumulate(/3),
    bitwise against: for each slot in rank order, first occurrence stores, later ones add, /3.
    records: the rows read from RowExchange's one-collective layout (rank blocks of
    [ids as 2*cap words | rows], rank_stride = cap*(d+2)) instead of one dense row table."""
    from lgcn_amd import _ffi

    lib = _ffi.load()
    U, I, W, cap = 500, 300, 3, 260
    N = U + I
    rng = np.random.default_rng(d)
    gens = [torch.randn(N, d, device=gpu) for _ in range(W)]
    ids_all, rows_all, expect_ids = [], [], []
    for r in range(W):
        rows_a = np.unique(rng.integers(0, N, 90)).astype(np.int32)
        negs = rng.integers(0, I, 120)
        first = np.zeros(len(negs), np.uint8)
        first[np.unique(negs, return_index=True)[1]] = 1
        skip = np.zeros(N, np.uint8)
        skip[rows_a] = 1
        ids, rows = _pack(lib, gens[r], U, d, torch.from_numpy(rows_a).to(gpu), torch.from_numpy(negs).to(gpu),
                          torch.from_numpy(first).to(gpu), torch.from_numpy(skip).to(gpu), cap, gpu)
        want = np.full(cap, -1, np.int64)
        want[:len(rows_a)] = rows_a
        for j, k in enumerate(negs):
            if first[j] and not skip[k + U]:
                want[len(rows_a) + j] = k + U
        assert np.array_equal(ids.cpu().numpy(), want)
        ok = torch.from_numpy(want >= 0).to(gpu)
        assert torch.equal(rows[ok], gens[r][ids[ok]])
        ids_all.append(ids)
        rows_all.append(rows)
    ids_all = torch.cat(ids_all)
    rows_all = torch.cat(rows_all)
    claim = torch.full((N,), 2**31 - 1, dtype=torch.int32, device=gpu)
    first = torch.empty(W * cap, dtype=torch.uint8, device=gpu)
    s = _ffi.stream_of(gpu)
    _ffi.check(lib.lgcn_rows_mark_first(ids_all.data_ptr(), W * cap, claim.data_ptr(), first.data_ptr(), s), "mf")
    assert torch.equal(claim, torch.full_like(claim, 2**31 - 1))
    g = torch.full((N, d), float("nan"), device=gpu)  # rows outside the union must stay untouched
    if records:
        blk = cap * (d + 2)
        rec = torch.full((W, blk), float("nan"), device=gpu)
        rec[:, :2 * cap] = ids_all.view(W, cap).view(torch.float32)
        rec[:, 2 * cap:] = rows_all.view(W, cap * d)
        rows_ptr, stride = rec.data_ptr() + 8 * cap, blk
    else:
        rows_ptr, stride = rows_all.data_ptr(), cap * d
    _ffi.check(lib.lgcn_rows_accumulate(ids_all.data_ptr(), rows_ptr, W, cap, stride, first.data_ptr(),
                                        g[:U].data_ptr(), g[U:].data_ptr(), U, d, float(W), s), "acc")
    ids_h = ids_all.cpu().numpy()
    rows_h = rows_all.cpu()
    ref = {}
    seen = set()
    first_ref = np.zeros(W * cap, np.uint8)
    for i, r in enumerate(ids_h):
        if r < 0:
            continue
        if r not in seen:
            seen.add(r)
            first_ref[i] = 1
            ref[r] = rows_h[i].clone()
        else:
            ref[r] = ref[r] + rows_h[i]
    assert np.array_equal(first.cpu().numpy(), first_ref)
    gh = g.cpu()
    for r, v in ref.items():
        assert torch.equal(gh[r], v / W), r
    outside = np.setdiff1d(np.arange(N), np.array(sorted(seen)))
    assert torch.isnan(gh[outside]).all()


@pytest.mark.parametrize("use_graphs", [False, True])
def test_exchange_world1_equals_plain_lazy_step(gpu, use_graphs):
    """With one rank the exchange must be a no-op: bitwise the plain row-lazy step."""
    import graphs
    from lgcn_amd import cluster as C
    from lgcn_amd import distributed as D
    from lgcn_amd.optim import RowLazyAdam
    from lgcn_amd.train_step import FusedTrainStep
    from models.light_gcn import LightGCN

    U, I, ei = graphs.subsampled(U=2000, I=1000, pairs=8000, seed=4)
    part = C.partition_nodes(ei, U + I, 8)
    batches = [_Batch(torch.from_numpy(x).to(gpu)) for x in C.intra_part_edges(ei, part, 8)]
    cap = D.exchange_capacity(batches, U)
    res = []
    for with_ex in (False, True):
        torch.manual_seed(0)
        m = LightGCN(U, I, num_layers=3, dim_h=64).to(gpu)
        opt = RowLazyAdam(m.user_embedding.weight.data, m.item_embedding.weight.data, lr=1e-2, max_grad_norm=1.0)
        ex = D.RowExchange(cap, U + I, 64, gpu, 1) if with_ex else None
        step = FusedTrainStep(m, opt, graphs=use_graphs, lazy=True, exchange=ex)
        losses = []
        for i in range(12):
            torch.cuda.manual_seed(100 + i)
            losses.append(step.step(batches[i % 8]).item())
        step.sync()
        res.append((losses, m.user_embedding.weight.detach().clone(), m.item_embedding.weight.detach().clone()))
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1], res[1][1]) and torch.equal(res[0][2], res[1][2])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("clip", [float("inf"), 1.0])
def test_dp2_row_exchange_matches_dense_allreduce(gpu, tmp_path, clip):
    """Two ranks (gloo, one GPU): the row-lazy step with the row-sparse exchange (eager and
    hipGraph) vs dense all_reduce + FusedAdam on the same batches and negatives. Without
    clipping: bitwise (W = 2: (a + b) / 2 either way). With clip 1: the norms sum the same
    squares in another order (see test_lazy_train_step_matches_dense_step) — losses to 1e-5,
    parameters to 1e-3 of their scale. Both ranks end bitwise identical in every variant."""
    port = str(_free_port())
    worker = str(ROOT / "tests" / "dp_exchange_worker.py")
    outs = [str(tmp_path / f"r{r}.pt") for r in range(2)]
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    procs = [subprocess.Popen([sys.executable, "-u", worker, str(r), "2", port, outs[r], str(clip)], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(2)]
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=100)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log
    res = [torch.load(o, weights_only=True) for o in outs]
    for name in ("dense", "lazy", "lazy_graphs", "owner", "owner_graphs"):
        assert torch.equal(res[0][name]["user"], res[1][name]["user"]), name
        assert torch.equal(res[0][name]["item"], res[1][name]["item"]), name
    for r in range(2):
        _check_owner_vs_replicated(res[r], clip)
    for r in range(2):
        d, lz, lg = res[r]["dense"], res[r]["lazy"], res[r]["lazy_graphs"]
        assert lz["losses"] == lg["losses"]
        assert torch.equal(lz["user"], lg["user"]) and torch.equal(lz["item"], lg["item"])
        if clip == float("inf"):
            assert d["losses"] == lz["losses"]
            assert torch.equal(d["user"], lz["user"]) and torch.equal(d["item"], lz["item"])
        else:
            for a, b in zip(d["losses"], lz["losses"]):
                assert abs(a - b) <= 1e-5 * max(1.0, abs(a))
            for k in ("user", "item"):
                assert (d[k] - lz[k]).abs().max().item() <= 1e-3 * d[k].abs().max().item()


def _check_owner_vs_replicated(res, clip):
    """Owner-sharded exchange vs the replicated one (both row-lazy): bitwise whenever the clip
    coefficient is exactly 1 (the same rank-ordered sums, the same updates and replays); with an
    active clip the two norms sum the same squares in another order (losses to 1e-5)."""
    lz, ow, og = res["lazy"], res["owner"], res["owner_graphs"]
    assert ow["losses"] == og["losses"]
    assert torch.equal(ow["user"], og["user"]) and torch.equal(ow["item"], og["item"])
    if clip == float("inf"):
        assert ow["losses"] == lz["losses"]
        assert torch.equal(ow["user"], lz["user"]) and torch.equal(ow["item"], lz["item"])
    else:
        for a, b in zip(lz["losses"], ow["losses"]):
            assert abs(a - b) <= 1e-5 * max(1.0, abs(a))


def _spawn(world, tmp_path, clip, variants, steps=12, npz=None, timeout=300, device_collectives=False):
    port = str(_free_port())
    worker = str(ROOT / "tests" / "dp_exchange_worker.py")
    tag = "dc" if device_collectives else "h"
    outs = [str(tmp_path / f"w{world}_{tag}_r{r}.pt") for r in range(world)]
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", DP_VARIANTS=variants, DP_STEPS=str(steps),
               OMP_NUM_THREADS="1", DP_DEVICE_COLLECTIVES="1" if device_collectives else "0")
    extra = [npz] if npz else []
    procs = [subprocess.Popen([sys.executable, "-u", worker, str(r), str(world), port, outs[r], str(clip), *extra],
                              env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(world)]
    logs = []
    try:
        for p in procs:
            logs.append(p.communicate(timeout=timeout)[0])
    except subprocess.TimeoutExpired:
        for q in procs:
            q.kill()
        raise
    for p, log in zip(procs, logs):
        # the first error lines of the rank's log (a HIP error's traceback starts well before its tail)
        first = "\n".join([ln for ln in log.splitlines() if "Error" in ln or "error" in ln][:8])
        assert p.returncode == 0, first + "\n...\n" + log[-2000:]
    return [torch.load(o, weights_only=True) for o in outs]


@pytest.mark.parametrize("clip", [float("inf"), 1.0])
def test_dp8_owner_exchange_matches_replicated(gpu, tmp_path, clip):
    """Eight ranks (gloo, one GPU), 16 steps with a different next batch each step: the
    owner-sharded optimizer (lgcn_amd.owner; gradient rows to their owners, rows fetched for the
    next step) == the replicated row exchange, bitwise without clipping; every rank ends with
    bitwise identical tables after sync(); the bytes each rank receives per step are printed."""
    res = _spawn(8, tmp_path, clip, "lazy,owner,owner_graphs", steps=16)
    for name in ("lazy", "owner", "owner_graphs"):
        for r in range(1, 8):
            assert torch.equal(res[0][name]["user"], res[r][name]["user"]), (name, r)
            assert torch.equal(res[0][name]["item"], res[r][name]["item"]), (name, r)
    for r in range(8):
        _check_owner_vs_replicated(res[r], clip)
    print(f"W=8 bytes received per rank per step: replicated {res[0]['lazy']['bytes_per_step'] / 1e6:.3f} MB, "
          f"owner {res[0]['owner']['bytes_per_step'] / 1e6:.3f} MB (cap {res[0]['cap']}, owner cap {res[0]['ocap']})")


def test_dp8_owner_exchange_dense_batches_matches_replicated(gpu, tmp_path):
    """Batches with many more triplets than items (each part's users draw every item several
    times as negatives — the planted graph's case): the owner-sharded exchange requests each
    distinct row once (lgcn_owner_pack_requests' claim, ABI 8), so its blocks are sized by the
    owner's items (owner_capacity(num_items=I)) rather than by its share of the triplets — and it
    stays bitwise the replicated exchange without clipping, with identical tables on every rank."""
    from lgcn_amd import cluster as C
    from lgcn_amd import synth
    from lgcn_amd.owner import owner_capacity

    g = synth.bipartite(640, 48, 9000, seed=5)
    U, I = g.num_users, g.num_items
    part = C.partition_nodes(g.edge_index, g.num_nodes, 8)
    lists = [x for x in C.intra_part_edges(g.edge_index, part, 8) if x.shape[1]]
    B = [int((x[0] < U).sum()) for x in lists]
    assert min(B) > I  # every batch draws more negatives than there are items
    batches = [_Batch(torch.from_numpy(x)) for x in lists]
    assert owner_capacity(batches, U, 8, num_items=I) < owner_capacity(batches, U, 8)
    npz = tmp_path / "dense_batches.npz"
    np.savez(npz, U=U, I=I, **{f"b{i}": x for i, x in enumerate(lists)})
    res = _spawn(8, tmp_path, float("inf"), "lazy,owner,owner_graphs", steps=16, npz=str(npz))
    for name in ("lazy", "owner", "owner_graphs"):
        for r in range(1, 8):
            assert torch.equal(res[0][name]["user"], res[r][name]["user"]), (name, r)
            assert torch.equal(res[0][name]["item"], res[r][name]["item"]), (name, r)
    for r in range(8):
        _check_owner_vs_replicated(res[r], float("inf"))
    print(f"dense batches (B {min(B)}-{max(B)} > I {I}), W=8: owner cap {res[0]['ocap']} "
          f"(without the item bound {owner_capacity(batches, U, 8)}), bytes received per rank per step: "
          f"replicated {res[0]['lazy']['bytes_per_step'] / 1e6:.3f} MB, owner {res[0]['owner']['bytes_per_step'] / 1e6:.3f} MB")


@pytest.mark.parametrize("world,clip", [(2, float("inf")), (4, float("inf")), (8, float("inf")), (2, 1.0)])
def test_hybrid_exchange_matches_replicated(gpu, tmp_path, world, clip):
    """HybridExchange (item gradient table all_reduced densely, users' rows as record blocks,
    every item row stepped each step): every rank ends bitwise identical, eager == graphs; at W = 2
    bitwise the replicated row exchange (a + b == b + a; the item rows a step leaves alone take
    Adam's zero-gradient step, bitwise the lazy replay); at W = 4 the item sums are the
    collective's order, not rank order — losses to 1e-5 of the replicated run's, tables within
    Adam's reach (2 lr per step) with all but 1e-3 of the elements inside the 1e-5 row bar. With
    clip 1 the clip norm sums the same squares in another order (every item row vs the union's
    rows): losses to 1e-5, tables within the same bar."""
    res = _spawn(world, tmp_path, clip, "lazy,hybrid,hybrid_graphs", steps=12)
    for name in ("lazy", "hybrid", "hybrid_graphs"):
        for r in range(1, world):
            assert torch.equal(res[0][name]["user"], res[r][name]["user"]), (name, r)
            assert torch.equal(res[0][name]["item"], res[r][name]["item"]), (name, r)
    lz, hy, hg = res[0]["lazy"], res[0]["hybrid"], res[0]["hybrid_graphs"]
    assert hy["losses"] == hg["losses"]
    assert torch.equal(hy["user"], hg["user"]) and torch.equal(hy["item"], hg["item"])
    if world == 2 and clip == float("inf"):
        assert hy["losses"] == lz["losses"]
        assert torch.equal(hy["user"], lz["user"]) and torch.equal(hy["item"], lz["item"])
        return
    for a, b in zip(lz["losses"], hy["losses"]):
        assert abs(a - b) <= 1e-5 * max(1.0, abs(a))
    for k in ("user", "item"):
        x, y = lz[k], hy[k]
        assert (x - y).abs().max().item() <= 2 * 1e-2 * 12
        scale = x.abs().amax(dim=1, keepdim=True).clamp_min(1e-30)
        off = ((x - y).abs() > 1e-5 * scale).float().mean().item()
        assert off <= 1e-3, (k, off)
    print(f"W={world} hybrid vs replicated: bytes received per rank per step {hy['bytes_per_step'] / 1e6:.3f} MB "
          f"vs {lz['bytes_per_step'] / 1e6:.3f} MB")


@pytest.mark.parametrize("world,clip", [(2, float("inf")), (2, 1.0), (4, 1.0)])
def test_column_sharded_graph_replay_matches_eager(gpu, tmp_path, world, clip):
    """Column-sharded training captured per batch as graphs cut at its two collectives
    (train_step._SegmentedGraph: the [B, 6] all_reduce and the norm partials' all_gather run
    eagerly between the replays) == the eager column-sharded step, bitwise, on every rank, over
    16 steps that revisit every batch (so each batch's captured graphs replay)."""
    res = _spawn(world, tmp_path, clip, "cols,cols_graphs", steps=16)
    for r in range(world):
        eager, graphs = res[r]["cols"], res[r]["cols_graphs"]
        assert eager["losses"] == graphs["losses"], r
        assert torch.equal(eager["user"], graphs["user"]) and torch.equal(eager["item"], graphs["item"]), r
        if r:
            assert eager["losses"] == res[0]["cols"]["losses"]  # every rank computes the full-width loss


@pytest.mark.parametrize("clip", [float("inf"), 1.0])
def test_dp_exchanges_device_collectives_equal_host_path(gpu, tmp_path, clip):
    """Four ranks (gloo, one GPU) down the RCCL branches (tuning device_collectives=True: RowExchange's
    all_gather_into_tensor, OwnerExchange's all_to_all_single / all_gather on CUDA tensors,
    ColumnGroup's device all_gather; the capacity all_reduces on device) == the same run through
    host memory, bitwise, for the replicated, owner-sharded and column-sharded modes (eager and
    graphs)."""
    variants = "lazy,lazy_graphs,owner,owner_graphs,cols,cols_graphs"
    host = _spawn(4, tmp_path, clip, variants, steps=12)
    dev = _spawn(4, tmp_path, clip, variants, steps=12, device_collectives=True)
    for r in range(4):
        for name in variants.split(","):
            assert host[r][name]["losses"] == dev[r][name]["losses"], (r, name)
            assert torch.equal(host[r][name]["user"], dev[r][name]["user"]), (r, name)
            assert torch.equal(host[r][name]["item"], dev[r][name]["item"]), (r, name)
