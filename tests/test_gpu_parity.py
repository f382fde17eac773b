"""HIP path vs the CPU oracle, through the C ABI (lgcn_amd → liblgcn.so).

Bars (BASELINE.json north_star): CSR index construction bit-exact; propagation
within 1e-5 relative fp32 PER ROW (tests/parity.py: max|Δ| of a row <= 1e-5 * max|ref| of that
row; the max elementwise relative error is reported with it). With every row unsplit (chunk >= max degree) the kernels add in exactly the
oracle's order, so forward and backward are also checked bit for bit.
"""
import numpy as np
import pytest
import torch

import graphs
from oracle import c_oracle
from oracle import lgconv_ref as R
from parity import assert_rows_close

pytestmark = pytest.mark.gpu


def _plan(ei, N, dev, chunk=None):
    from lgcn_amd.plan import DEFAULT_CHUNK, PropagationPlan

    return PropagationPlan(torch.from_numpy(ei).to(dev), N, chunk or DEFAULT_CHUNK)


@pytest.mark.parametrize("name", list(graphs.ALL))
def test_csr_bit_exact(gpu, name):
    U, I, ei = graphs.ALL[name]()
    N = U + I
    plan = _plan(ei, N, gpu)
    for direction, key, other in ((plan.fwd, ei[1], ei[0]), (plan.bwd, ei[0], ei[1])):
        rp, col, eid = c_oracle.csr_build(key, other, N)
        assert np.array_equal(direction.rowptr.cpu().numpy(), rp)
        assert np.array_equal(direction.col.cpu().numpy(), col)
        assert np.array_equal(direction.eid.cpu().numpy(), eid)
    # gcn_norm weights, bit-exact, in CSR order
    dis, w_edge = c_oracle.gcn_norm(ei, N)
    assert np.array_equal(plan.dis.cpu().numpy(), dis)
    assert np.array_equal(plan.fwd.val.cpu().numpy(), w_edge[plan.fwd.eid.cpu().numpy()])
    assert np.array_equal(plan.bwd.val.cpu().numpy(), w_edge[plan.bwd.eid.cpu().numpy()])


@pytest.mark.parametrize("chunk", [1, 3, 16, 256])
def test_schedule_covers_rows(gpu, chunk):
    U, I, ei = graphs.hub()
    N = U + I
    plan = _plan(ei, N, gpu, chunk)
    f = plan.fwd
    items = f.item_table().cpu().numpy()
    rowptr = f.rowptr.cpu().numpy()
    deg = np.diff(rowptr)
    assert f.n_items == sum(max(1, -(-int(x) // chunk)) for x in deg)
    # longest first
    assert np.all(np.diff(items[:, 1]) <= 0)
    covered = np.zeros(rowptr[-1], np.int64)
    whole_rows = items[items[:, 2] >= 0, 2]
    assert len(set(whole_rows.tolist())) == len(whole_rows)
    for beg, ln, dst in items:
        covered[beg:beg + ln] += 1
        assert ln <= chunk
    assert np.all(covered == 1)
    splits = f.splits[: f.n_splits].cpu().numpy()
    assert set(whole_rows.tolist()) | set(splits[:, 0].tolist()) == set(range(N))
    assert f.n_partials == int(splits[:, 2].sum()) if f.n_splits else f.n_partials == 0


@pytest.mark.parametrize("name", list(graphs.ALL))
@pytest.mark.parametrize("K", [0, 1, 2, 3, 4])
def test_forward_backward(gpu, name, K):
    from models.light_gcn import LightGCN

    U, I, ei = graphs.ALL[name]()
    d = 64
    uw, iw = graphs.embeddings(U, I, d, seed=K)
    model = LightGCN(U, I, num_layers=K, dim_h=d).to(gpu)
    with torch.no_grad():
        model.user_embedding.weight.copy_(torch.from_numpy(uw))
        model.item_embedding.weight.copy_(torch.from_numpy(iw))
    et = torch.from_numpy(ei).to(gpu)
    users, items = model(et)
    ru, ri = c_oracle.lightgcn_forward(uw, iw, ei, K)
    assert users.shape == (U, d) and items.shape == (I, d)
    assert_rows_close(users.detach().cpu().numpy(), ru)
    assert_rows_close(items.detach().cpu().numpy(), ri)

    dF = np.random.default_rng(K + 11).standard_normal((U + I, d)).astype(np.float32)
    (torch.cat([users, items]) * torch.from_numpy(dF).to(gpu)).sum().backward()
    gu, gi = c_oracle.lightgcn_backward(dF, ei, U, K)
    assert_rows_close(model.user_embedding.weight.grad.cpu().numpy(), gu)
    assert_rows_close(model.item_embedding.weight.grad.cpu().numpy(), gi)


@pytest.mark.parametrize("name", ["sym", "subsampled", "shuffled", "hub"])
def test_bit_exact_unsplit(gpu, name):
    """chunk >= max degree: every row is one item, summed in CSR order with mul-then-add —
    bitwise the reference CPU scatter_add_ result, forward and backward."""
    from lgcn_amd import propagate_backward, propagate_forward

    U, I, ei = graphs.ALL[name]()
    N, K, d = U + I, 3, 64
    plan = _plan(ei, N, gpu, chunk=1 << 20)
    assert plan.fwd.n_splits == 0
    uw, iw = graphs.embeddings(U, I, d, seed=5)
    out = propagate_forward(torch.from_numpy(uw).to(gpu), torch.from_numpy(iw).to(gpu), plan, K)
    ru, ri = c_oracle.lightgcn_forward(uw, iw, ei, K)
    assert np.array_equal(out.cpu().numpy(), np.concatenate([ru, ri]))
    dF = np.random.default_rng(3).standard_normal((N, d)).astype(np.float32)
    gu, gi = propagate_backward(torch.from_numpy(dF).to(gpu), plan, U, K)
    ou, oi = c_oracle.lightgcn_backward(dF, ei, U, K)
    assert np.array_equal(gu.cpu().numpy(), ou)
    assert np.array_equal(gi.cpu().numpy(), oi)


@pytest.mark.parametrize("d", [4, 16, 64, 128, 256, 512, 1024])
@pytest.mark.parametrize("tail", [1, 0])
def test_tail_paths_bit_exact(gpu, tune, d, tail):
    """Both item-pass tail paths (tuning spmm_tail 1 = predicated tail forced on, 0 = forced
    off; the default picks per width and launch size) add in CSR order: unsplit rows of every
    length 1..max are bitwise the oracle, forward and backward."""
    from lgcn_amd import propagate_backward, propagate_forward

    tune(spmm_tail=tail)
    U, I, ei = graphs.sym()
    N, K = U + I, 2
    plan = _plan(ei, N, gpu, chunk=1 << 20)
    uw, iw = graphs.embeddings(U, I, d, seed=d)
    out = propagate_forward(torch.from_numpy(uw).to(gpu), torch.from_numpy(iw).to(gpu), plan, K)
    ru, ri = c_oracle.lightgcn_forward(uw, iw, ei, K)
    assert np.array_equal(out.cpu().numpy(), np.concatenate([ru, ri]))
    dF = np.random.default_rng(d).standard_normal((N, d)).astype(np.float32)
    gu, gi = propagate_backward(torch.from_numpy(dF).to(gpu), plan, U, K)
    ou, oi = c_oracle.lightgcn_backward(dF, ei, U, K)
    assert np.array_equal(gu.cpu().numpy(), ou)
    assert np.array_equal(gi.cpu().numpy(), oi)


@pytest.mark.parametrize("d", [4, 16, 64, 128, 256, 512, 1024])
@pytest.mark.parametrize("chunk", [3, 32])
def test_blocksplit_equals_items_plus_combine(gpu, d, chunk):
    """lgcn_spmm_blocksplit (split rows summed by one workgroup each, one launch) is bitwise the
    item pass + combine pair, forward and backward, with split rows of 2..700 chunks; and both
    are within 1e-5 of the oracle."""
    from lgcn_amd import propagate_backward, propagate_forward

    U, I, ei = graphs.hub()
    N, K = U + I, 2
    plan = _plan(ei, N, gpu, chunk=chunk)
    assert plan.fwd.n_splits > 0 and plan.bwd.n_splits > 0
    uw, iw = graphs.embeddings(U, I, d, seed=d)
    dF = np.random.default_rng(d).standard_normal((N, d)).astype(np.float32)
    res = []
    for bs in (False, True):
        plan.fwd.block_split = plan.bwd.block_split = bs
        out = propagate_forward(torch.from_numpy(uw).to(gpu), torch.from_numpy(iw).to(gpu), plan, K)
        gu, gi = propagate_backward(torch.from_numpy(dF).to(gpu), plan, U, K)
        res.append((out.cpu(), gu.cpu(), gi.cpu()))
    for a, b in zip(*res):
        assert torch.equal(a, b)
    ru, ri = c_oracle.lightgcn_forward(uw, iw, ei, K)
    assert_rows_close(res[1][0].numpy(), np.concatenate([ru, ri]))


def test_blocksplit_argument_errors(gpu):
    """The one-launch entry point refuses split rows without their chunk list, and widths the
    vector kernels do not cover (no silent fallback)."""
    from lgcn_amd import _ffi

    U, I, ei = graphs.hub()
    N = U + I
    plan = _plan(ei, N, gpu, chunk=8)
    f = plan.fwd
    rows, n_rows, chunks = f.block_lists()
    lib = _ffi.load()
    s = _ffi.stream_of(gpu)
    common = (rows.data_ptr(), n_rows, f.splits.data_ptr(), f.n_splits, f.col.data_ptr(), f.val.data_ptr(), N)
    for d, ch, code in ((16, None, -1), (12, chunks.data_ptr(), -3)):
        x = torch.zeros((N, d), device=gpu)
        y = torch.zeros((N, d), device=gpu)
        rc = lib.lgcn_spmm_blocksplit(*common, d, x.data_ptr(), None, N, None, None, N, None, y.data_ptr(), None, N,
                                      None, _ffi.EPI_STORE, 1.0, 1.0, s, ch)
        assert rc == code, lib.lgcn_last_error()


@pytest.mark.parametrize("d", [3, 4, 8, 16, 32, 96, 128, 256, 512, 200])
def test_widths(gpu, d):
    """Vector kernels (d in {4..1024} powers of two) and the scalar path (other d)."""
    from lgcn_amd import propagate_backward, propagate_forward

    U, I, ei = graphs.hub(U=600, I=40)
    N, K = U + I, 2
    plan = _plan(ei, N, gpu, chunk=64)
    uw, iw = graphs.embeddings(U, I, d, seed=d)
    out = propagate_forward(torch.from_numpy(uw).to(gpu), torch.from_numpy(iw).to(gpu), plan, K)
    ru, ri = c_oracle.lightgcn_forward(uw, iw, ei, K)
    assert_rows_close(out.cpu().numpy(), np.concatenate([ru, ri]))
    dF = np.random.default_rng(d).standard_normal((N, d)).astype(np.float32)
    gu, gi = propagate_backward(torch.from_numpy(dF).to(gpu), plan, U, K)
    ou, oi = c_oracle.lightgcn_backward(dF, ei, U, K)
    assert_rows_close(np.concatenate([gu.cpu().numpy(), gi.cpu().numpy()]), np.concatenate([ou, oi]))


def test_lgconv_operator(gpu):
    """The single-layer operator boundary: LGConv()(x, edge_index) and its gradient."""
    import lgcn_amd

    U, I, ei = graphs.subsampled()
    N, d = U + I, 64
    x = np.random.default_rng(0).standard_normal((N, d)).astype(np.float32)
    xt = torch.from_numpy(x).to(gpu).requires_grad_(True)
    conv = lgcn_amd.LGConv()
    y = conv(x=xt, edge_index=torch.from_numpy(ei).to(gpu))
    w = R.gcn_norm(ei, N)
    assert_rows_close(y.detach().cpu().numpy(), R.lgconv(x, ei, w))
    dy = np.random.default_rng(1).standard_normal((N, d)).astype(np.float32)
    y.backward(torch.from_numpy(dy).to(gpu))
    assert_rows_close(xt.grad.cpu().numpy(), R.lgconv_transposed(dy, ei, w))


def test_empty_edges(gpu):
    from models.light_gcn import LightGCN

    U, I, d, K = 7, 5, 64, 3
    model = LightGCN(U, I, num_layers=K, dim_h=d).to(gpu)
    ei = torch.empty((2, 0), dtype=torch.int64, device=gpu)
    users, items = model(ei)
    uw = model.user_embedding.weight.detach().cpu().numpy()
    iw = model.item_embedding.weight.detach().cpu().numpy()
    ru, ri = c_oracle.lightgcn_forward(uw, iw, np.zeros((2, 0), np.int64), K)
    assert np.array_equal(users.detach().cpu().numpy(), ru)
    assert np.array_equal(items.detach().cpu().numpy(), ri)
    (users.sum() + items.sum()).backward()
    assert torch.all(model.user_embedding.weight.grad == (1.0 * np.float32(0.25)) / 4)


def test_out_of_range_ids_raise(gpu):
    from models.light_gcn import LightGCN

    model = LightGCN(4, 3, num_layers=2, dim_h=8).to(gpu)
    bad = torch.tensor([[0, 1], [4, 7]], dtype=torch.int64, device=gpu)  # 7 >= N
    with pytest.raises(IndexError):
        model(bad)


def test_deterministic(gpu):
    from lgcn_amd import propagate_forward

    U, I, ei = graphs.hub()
    plan = _plan(ei, U + I, gpu, chunk=32)
    uw, iw = graphs.embeddings(U, I, 64)
    a = propagate_forward(torch.from_numpy(uw).to(gpu), torch.from_numpy(iw).to(gpu), plan, 3)
    b = propagate_forward(torch.from_numpy(uw).to(gpu), torch.from_numpy(iw).to(gpu), plan, 3)
    assert torch.equal(a, b)


def test_plan_cache_reuse_and_invalidation(gpu):
    from models.light_gcn import LightGCN

    U, I, ei = graphs.sym()
    model = LightGCN(U, I, num_layers=2, dim_h=16).to(gpu)
    et = torch.from_numpy(ei).to(gpu)
    p1 = model.plan_for(et)
    assert model.plan_for(et) is p1
    # plans are found by content (lgcn_amd._cache): a new tensor of the same edges — what the
    # reference's PyG loader collates every epoch — gets the same plan
    assert model.plan_for(et.clone()) is p1
    et[0, 0] = et[0, 0]  # in-place write bumps the version counter: re-keyed, the same edges
    assert model.plan_for(et) is p1
    et[:, [0, 1]] = et[:, [1, 0]].clone()  # an in-place change of the edge list: a new plan
    assert model.plan_for(et) is not p1


def test_ml25m_scaled_parity(gpu):
    """A 5%-scale ML-25M-shaped graph (E ≈ 1.2M) with the default schedule."""
    from lgcn_amd import synth
    from models.light_gcn import LightGCN

    g = synth.ml25m_shaped(seed=3, scale=0.05)
    U, I, K, d = g.num_users, g.num_items, 3, 64
    model = LightGCN(U, I, num_layers=K, dim_h=d).to(gpu)
    users, items = model(torch.from_numpy(g.edge_index).to(gpu))
    uw = model.user_embedding.weight.detach().cpu().numpy()
    iw = model.item_embedding.weight.detach().cpu().numpy()
    ru, ri = c_oracle.lightgcn_forward(uw, iw, g.edge_index, K)
    assert_rows_close(users.detach().cpu().numpy(), ru)
    assert_rows_close(items.detach().cpu().numpy(), ri)
