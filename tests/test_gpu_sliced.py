"""The source-sliced schedule (lgcn_amd.sliced, lgcn_spmm_run): one launch per source slice,
row sums carried between launches through the running buffer. Forced on small graphs with
tuning slice_mb and a short chunk (so hub rows take the chunk + combine path too), against the C
oracle: within 1e-5 everywhere, and bitwise on every row summed as one sequential chain."""
import numpy as np
import pytest
import torch

import graphs
from oracle import c_oracle
from parity import assert_rows_close

pytestmark = pytest.mark.gpu


def _plan(ei, N, dev, U, chunk):
    from lgcn_amd.plan import PropagationPlan

    return PropagationPlan(torch.from_numpy(ei).to(dev), N, chunk, side_split=U)


@pytest.fixture
def force_slices(tune):
    def set_mb(mb):
        tune(slice_mb=float(mb))
    return set_mb


def _hub_mask(sched, N):
    m = np.zeros(N, bool)
    m[sched.splits[: sched.n_splits, 0].cpu().numpy()] = True
    return m


@pytest.mark.parametrize("name", ["sym", "subsampled", "hub", "isolated"])
@pytest.mark.parametrize("K", [1, 2, 3, 4])
def test_sliced_forward_backward(gpu, force_slices, name, K):
    from lgcn_amd import propagate_backward, propagate_forward
    from lgcn_amd.sliced import SlicedDirection

    U, I, ei = graphs.ALL[name]()
    N, d = U + I, 64
    force_slices(0.005)  # ~20 rows of width 64 per slice
    plan = _plan(ei, N, gpu, U, chunk=8)
    sched = plan.schedule("fwd", d)
    assert isinstance(sched, SlicedDirection) and len(sched.launches) > 4
    uw, iw = graphs.embeddings(U, I, d, seed=K)
    out = propagate_forward(torch.from_numpy(uw).to(gpu), torch.from_numpy(iw).to(gpu), plan, K).cpu().numpy()
    ru, ri = c_oracle.lightgcn_forward(uw, iw, ei, K)
    ref = np.concatenate([ru, ri])
    assert_rows_close(out, ref)
    dF = np.random.default_rng(K).standard_normal((N, d)).astype(np.float32)
    gu, gi = propagate_backward(torch.from_numpy(dF).to(gpu), plan, U, K)
    ou, oi = c_oracle.lightgcn_backward(dF, ei, U, K)
    assert_rows_close(np.concatenate([gu.cpu().numpy(), gi.cpu().numpy()]), np.concatenate([ou, oi]))


@pytest.mark.parametrize("name", ["sym", "subsampled", "hub"])
@pytest.mark.parametrize("mb", [0.002, 0.01, 0.05])
def test_sliced_layer_bitwise_on_chained_rows(gpu, force_slices, name, mb):
    """One layer (the LGConv operator): rows outside the hub set are bitwise the oracle —
    their sequential CSR-order chain survives being split across slice launches."""
    from lgcn_amd.propagate import lgconv_backward, lgconv_forward

    U, I, ei = graphs.ALL[name]()
    N, d = U + I, 64
    force_slices(mb)
    plan = _plan(ei, N, gpu, U, chunk=16)
    x = np.random.default_rng(4).standard_normal((N, d)).astype(np.float32)
    y = lgconv_forward(torch.from_numpy(x).to(gpu), plan).cpu().numpy()
    _, w = c_oracle.gcn_norm(ei, N)
    ref = c_oracle.lgconv(x, ei, w)
    hub = _hub_mask(plan.schedule("fwd", d), N)
    assert np.array_equal(y[~hub], ref[~hub])
    assert_rows_close(y, ref)
    # transposed operator (autograd backward of one layer)
    gy = lgconv_backward(torch.from_numpy(x).to(gpu), plan).cpu().numpy()
    ref_t = c_oracle.lgconv(x, ei[::-1].copy(), w)
    hub_t = _hub_mask(plan.schedule("bwd", d), N)
    assert np.array_equal(gy[~hub_t], ref_t[~hub_t])


@pytest.mark.parametrize("d", [8, 32, 128, 256])
def test_sliced_widths_and_default_agree(gpu, force_slices, d):
    """Sliced and plain schedules agree bitwise on rows that both sum as one chain."""
    from lgcn_amd.propagate import lgconv_forward

    U, I, ei = graphs.hub(U=700, I=60)
    N = U + I
    x = torch.from_numpy(np.random.default_rng(d).standard_normal((N, d)).astype(np.float32)).to(gpu)
    force_slices(0)
    plain = _plan(ei, N, gpu, U, chunk=32)
    a = lgconv_forward(x, plain).cpu().numpy()
    force_slices(0.003)
    sliced = _plan(ei, N, gpu, U, chunk=32)
    b = lgconv_forward(x, sliced).cpu().numpy()
    split_plain = np.zeros(N, bool)
    split_plain[plain.fwd.splits[: plain.fwd.n_splits, 0].cpu().numpy()] = True
    ok = ~split_plain & ~_hub_mask(sliced.schedule("fwd", d), N)
    assert ok.sum() > N // 2
    assert np.array_equal(a[ok], b[ok])
    assert_rows_close(b, a)


def test_sliced_schedule_covers_edges_once(gpu, force_slices):
    from lgcn_amd.sliced import ITEM_FIRST, ITEM_LAST

    U, I, ei = graphs.hub()
    N = U + I
    force_slices(0.004)
    plan = _plan(ei, N, gpu, U, chunk=8)
    sd = plan.schedule("fwd", 64)
    E = ei.shape[1]
    cover = np.zeros(E, np.int64)
    first = np.zeros(N, np.int64)
    last = np.zeros(N, np.int64)
    for items, n in sd.launches:
        it = items.cpu().numpy()
        for beg, word in it:
            ln = int(word & 0xFFFFFFFF)
            dst = int(np.int64(word) >> 32)
            if dst >= 0:
                first[dst] += bool(ln & ITEM_FIRST)
                last[dst] += bool(ln & ITEM_LAST)
                ln &= 0x1FFFFFFF
            cover[beg:beg + ln] += 1
    assert np.all(cover == 1)
    hub = _hub_mask(sd, N)
    assert np.all(first[~hub] == 1) and np.all(last[~hub] == 1)
    assert np.all(first[hub] == 0) and np.all(last[hub] == 0)


def test_uncoalesced_edges_fall_back_to_plain_schedule(gpu, force_slices):
    """Rows whose neighbours are not ascending (a shuffled edge_index) cannot chain through the
    slices in CSR order, so the plain schedule runs; results still match the oracle."""
    from lgcn_amd import propagate_forward
    from lgcn_amd.plan import CsrDirection

    U, I, ei = graphs.shuffled()
    N, d = U + I, 64
    force_slices(0.005)
    plan = _plan(ei, N, gpu, U, chunk=8)
    assert isinstance(plan.schedule("fwd", d), CsrDirection)
    uw, iw = graphs.embeddings(U, I, d, seed=1)
    out = propagate_forward(torch.from_numpy(uw).to(gpu), torch.from_numpy(iw).to(gpu), plan, 3).cpu().numpy()
    ru, ri = c_oracle.lightgcn_forward(uw, iw, ei, 3)
    assert_rows_close(out, np.concatenate([ru, ri]))




@pytest.mark.parametrize("d,cms", [(64, [1, 2, 4]), (32, [1, 4, 8]), (16, [2, 8, 16]), (8, [4, 16, 32])])
@pytest.mark.parametrize("sliced", [True, False])
def test_index_rounds_bitwise(gpu, force_slices, tune, d, cms, sliced):
    """Index load rounds (tuning spmm_index_rounds batches of col/val per load round) only change how many
    indices a lane group loads at once, never the adds: every round size gives the same floats,
    on the sliced and the plain schedule, and matches the oracle."""
    from lgcn_amd.propagate import lgconv_forward

    U, I, ei = graphs.hub(U=900, I=80)
    N = U + I
    force_slices(0.004 if sliced else 0)
    plan = _plan(ei, N, gpu, U, chunk=24)
    x = torch.from_numpy(np.random.default_rng(d).standard_normal((N, d)).astype(np.float32)).to(gpu)
    outs = []
    for cm in cms:
        tune(spmm_index_rounds=cm)
        outs.append(lgconv_forward(x, plan).cpu().numpy())
    for o in outs[1:]:
        assert np.array_equal(o, outs[0])
    _, w = c_oracle.gcn_norm(ei, N)
    assert_rows_close(outs[0], c_oracle.lgconv(x.cpu().numpy(), ei, w))


@pytest.mark.parametrize("name", ["sym", "subsampled", "hub"])
@pytest.mark.parametrize("K,d,mb", [(2, 64, 0.005), (3, 64, 0.01), (4, 16, 0.002), (5, 128, 0.02), (3, 256, 0.05)])
def test_sliced_ride_bitwise(gpu, force_slices, tune, name, K, d, mb):
    """The riding-combine forward (lgcn_spmm_run_slices_ride: slice groups alternating per layer,
    each group's split rows combined inside the next group's first launch, partials double-buffered
    by layer parity, one combine launch at the end) is bitwise the per-layer slices + combine — run
    twice to show nothing carries over between calls."""
    from lgcn_amd import propagate_forward
    from lgcn_amd.sliced import ride_layout

    U, I, ei = graphs.ALL[name]()
    N = U + I
    force_slices(mb)
    plan = _plan(ei, N, gpu, U, chunk=8)
    sched = plan.schedule("fwd", d)
    r = ride_layout(sched, U)
    assert r is not None and 0 < r["nu"] < len(sched.launches)
    assert r["users"][1] + r["items"][1] == sched.n_splits
    uw, iw = graphs.embeddings(U, I, d, seed=K + d)
    uw_t, iw_t = torch.from_numpy(uw).to(gpu), torch.from_numpy(iw).to(gpu)
    tune(slice_ride=False)
    want = propagate_forward(uw_t, iw_t, plan, K).cpu()
    tune(slice_ride=True)
    for _ in range(2):
        got = propagate_forward(uw_t, iw_t, plan, K).cpu()
        assert torch.equal(got, want)
    ru, ri = c_oracle.lightgcn_forward(uw, iw, ei, K)
    assert_rows_close(got.numpy(), np.concatenate([ru, ri]))


def test_sliced_ride_off_for_non_bipartite(gpu, force_slices):
    """A user-user edge breaks the two groups' disjointness: no riding layout, and the forward
    (per-layer combines) still matches the oracle."""
    from lgcn_amd import propagate_forward
    from lgcn_amd.sliced import SlicedDirection, ride_layout

    U, I, ei = graphs.sym()
    ei = np.concatenate([ei, np.array([[1, 2], [2, 1]], dtype=ei.dtype)], axis=1)
    ei = np.ascontiguousarray(ei[:, np.lexsort((ei[0], ei[1]))])  # coalesced: the sliced schedule needs it
    N, d, K = U + I, 64, 3
    force_slices(0.005)
    plan = _plan(ei, N, gpu, U, chunk=8)
    sched = plan.schedule("fwd", d)
    assert isinstance(sched, SlicedDirection) and ride_layout(sched, U) is None
    uw, iw = graphs.embeddings(U, I, d, seed=1)
    out = propagate_forward(torch.from_numpy(uw).to(gpu), torch.from_numpy(iw).to(gpu), plan, K).cpu().numpy()
    ru, ri = c_oracle.lightgcn_forward(uw, iw, ei, K)
    assert_rows_close(out, np.concatenate([ru, ri]))
