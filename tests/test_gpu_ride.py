"""The Adam catch-up riding in block-split launches (lgcn_spmm_blocksplit_ride, lgcn_adam_ride_t;
FusedTrainStep._ride): the next batch's user rows advanced by extra workgroups of the current
step's propagation launches.

* ABI level: the pass's rows are bitwise the plain launch's; each ride row is bitwise what
  lgcn_row_adam's catch-up gives it for the same target step (never past the step in progress,
  at most max_replays per launch); skipped rows untouched.
* Training: whole epochs of row-lazy steps with the riding catch-up — with the true next batch, a
  wrong one, and a replay budget too small to finish — are bitwise the steps without it (losses
  and tables after the epoch flush), eager and hipGraph-replayed, with and without clipping.
Reference: utils/train_test.py:95-96 (Adam over both tables every step)."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


class _Batch:
    def __init__(self, ei):
        self.edge_index = ei


def _tables(gpu, U, I, d, seed=0):
    from lgcn_amd.optim import RowLazyAdam

    g = torch.Generator(device=gpu).manual_seed(seed)
    uw = torch.randn(U, d, device=gpu, generator=g) * 0.1
    iw = torch.randn(I, d, device=gpu, generator=g) * 0.1
    opt = RowLazyAdam(uw, iw, lr=1e-2, max_steps=256)
    for t in (*opt.m, *opt.v):
        t.copy_(torch.rand(t.shape, device=gpu, generator=g) * 1e-3)
    return opt


def _ride_rec(opt, rows, skip, R, U):
    from lgcn_amd import _ffi

    return _ffi.AdamRide(rows.data_ptr(), rows.numel(), skip.data_ptr() if skip is not None else None,
                         opt.uw.data_ptr(), opt.iw.data_ptr(), opt.m[0].data_ptr(), opt.m[1].data_ptr(),
                         opt.v[0].data_ptr(), opt.v[1].data_ptr(), U, opt.last.data_ptr(), opt.step_dev.data_ptr(),
                         opt.consts.data_ptr(), 1 - opt.betas[0], opt.betas[1], opt.eps, R)


def _snap(opt):
    return [t.clone() for t in (opt.uw, opt.iw, *opt.m, *opt.v, opt.last)]


@pytest.mark.parametrize("d", [16, 64, 128])
@pytest.mark.parametrize("R", [3, 40])
def test_blocksplit_ride_rows_equal_row_adam_catch_up(gpu, d, R):
    import graphs

    from lgcn_amd import _ffi
    from lgcn_amd.plan import PropagationPlan
    from lgcn_amd.propagate import spmm

    U, I, ei = graphs.subsampled(U=600, I=300, pairs=3000, seed=2)
    N = U + I
    plan = PropagationPlan(torch.from_numpy(ei).to(gpu), N, 32, side_split=U, touched_only=True)
    f = plan.schedule("fwd", d)
    assert f.block_split
    x = torch.randn(N, d, device=gpu, generator=torch.Generator(device=gpu).manual_seed(d))
    T = 30
    opt = _tables(gpu, U, I, d, seed=d)
    opt.step_dev.fill_(T)
    opt.steps = T
    rng = np.random.default_rng(R + d)
    last0 = torch.from_numpy(rng.integers(T - 25, T + 1, N).astype(np.int32)).to(gpu)
    opt.last.copy_(last0)
    rows = torch.from_numpy(rng.choice(U, 200, replace=False).astype(np.int32)).to(gpu)
    skip = torch.zeros(N, dtype=torch.uint8, device=gpu)
    skip[rows[::5].long()] = 1  # every fifth listed row belongs to the "current batch": left alone
    before = _snap(opt)
    # the pass alone, and the pass with the ride: the same rows
    outs = []
    for ride in (None, _ride_rec(opt, rows, skip, R, U)):
        acc = torch.zeros(N, d, device=gpu)
        spmm(f, N, d, (x, None, N), None, (acc, None, N), None, _ffi.EPI_STORE, ride=ride)
        outs.append(acc)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    got = _snap(opt)
    # the reference: lgcn_row_adam's catch-up (mode 0) of the unskipped rows to each row's target
    # min(last + R, T + 1), grouped by target (the catch-up takes one target per launch)
    ref = _tables(gpu, U, I, d, seed=d)
    for dst, src in zip((ref.uw, ref.iw, *ref.m, *ref.v, ref.last), before):
        dst.copy_(src)
    lst = last0[rows.long()].long()
    target = torch.minimum(lst + R, torch.full_like(lst, T + 1))
    live = (skip[rows.long()] == 0) & (target > lst)
    for t in sorted(set(target[live].tolist())):
        sel = rows[live & (target == t)].contiguous()
        ref.step_dev.fill_(t)
        ref.claim.fill_(-1)
        ref.catch_up(sel)
    torch.cuda.synchronize()
    for a, b in zip(got, _snap(ref)):
        assert torch.equal(a, b)
    # rows outside the list, and the skipped ones, untouched
    untouched = torch.ones(N, dtype=torch.bool, device=gpu)
    untouched[rows[live].long()] = False
    assert torch.equal(got[-1][untouched], before[-1][untouched])
    assert int(live.sum()) > 0


def test_blocksplit_ride_argument_errors(gpu):
    from lgcn_amd import _ffi

    lib = _ffi.load()
    bad = _ffi.AdamRide()
    bad.n_rows = 4  # rows NULL
    rc = lib.lgcn_spmm_blocksplit_ride(None, 0, None, 0, None, None, 8, 16, None, None, 8, None, None, 8, None,
                                       None, None, 8, None, 4, 1.0, 1.0, None, None, ctypes.byref(bad))
    assert rc != 0


@pytest.mark.parametrize("use_graphs", [False, True])
@pytest.mark.parametrize("clip", [float("inf"), 1.0])
@pytest.mark.parametrize("nxt", ["true", "wrong", "short"])
def test_lazy_steps_with_riding_catch_up_bitwise(gpu, tune, use_graphs, clip, nxt):
    """Three epochs of 8 Cluster-GCN batches, flushed at each epoch end (bench.py's loop): the
    riding catch-up on (true next batch; a wrong next batch; 1 replay per launch, so most rows are
    still behind at their step) is bitwise the run without it."""
    from lgcn_amd import cluster as C
    from lgcn_amd.optim import RowLazyAdam
    from lgcn_amd.train_step import FusedTrainStep
    from models.light_gcn import LightGCN

    import graphs

    U, I, ei = graphs.subsampled(U=2000, I=1000, pairs=8000, seed=4)
    part = C.partition_nodes(ei, U + I, 8)
    batches = [_Batch(torch.from_numpy(x).to(gpu)) for x in C.intra_part_edges(ei, part, 8)]
    rng = np.random.default_rng(3)
    res = []
    for ride in (False, True):
        tune(adam_ride_replays=(1 if nxt == "short" else 8) if ride else 0)
        torch.manual_seed(0)
        m = LightGCN(U, I, num_layers=3, dim_h=64).to(gpu)
        opt = RowLazyAdam(m.user_embedding.weight.data, m.item_embedding.weight.data, lr=1e-2, max_grad_norm=clip)
        step = FusedTrainStep(m, opt, graphs=use_graphs, lazy=True)
        losses = []
        for e in range(3):
            for i in range(8):
                torch.cuda.manual_seed(100 + 8 * e + i)
                if nxt == "wrong":
                    nb = batches[int(rng.integers(0, 8))]
                else:
                    nb = batches[i + 1] if i + 1 < 8 else None
                losses.append(step.step(batches[i], nb).item())
            step.sync()
        res.append((losses, m.user_embedding.weight.detach().clone(), m.item_embedding.weight.detach().clone(),
                    opt.m[0].clone(), opt.v[1].clone()))
        if ride:
            assert any(getattr(st, "_ride_cache", None) is not None for st in step._states.values())
    assert res[0][0] == res[1][0]
    for a, b in zip(res[0][1:], res[1][1:]):
        assert torch.equal(a, b)
