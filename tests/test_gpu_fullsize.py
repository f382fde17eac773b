"""Parity at BASELINE.json's full C2 size (ML-25M-shaped, E = 24.9M, K=3, d=64):
the whole forward against the C oracle (single-threaded, ~1 min of CPU), plus size-independent
properties of the propagation operator (adjointness and linearity)."""
import numpy as np
import pytest
import torch

from oracle import c_oracle
from parity import assert_rows_close

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c2(gpu):
    from lgcn_amd import synth
    from lgcn_amd.plan import PropagationPlan

    g = synth.ml25m_shaped(seed=0)
    ei = torch.from_numpy(g.edge_index).to(gpu)
    plan = PropagationPlan(ei, g.num_nodes, side_split=g.num_users)
    return g, plan


def test_c2_full_forward_matches_oracle(gpu, c2):
    from lgcn_amd import propagate_forward

    g, plan = c2
    rng = np.random.default_rng(0)
    uw = (rng.standard_normal((g.num_users, 64)) * 0.01).astype(np.float32)
    iw = (rng.standard_normal((g.num_items, 64)) * 0.01).astype(np.float32)
    out = propagate_forward(torch.from_numpy(uw).to(gpu), torch.from_numpy(iw).to(gpu), plan, 3).cpu().numpy()
    ru, ri = c_oracle.lightgcn_forward(uw, iw, g.edge_index, 3)
    ref = np.concatenate([ru, ri])
    assert_rows_close(out, ref)


@pytest.mark.parametrize("d", [8, 16, 32])
def test_c2_column_share_widths_match_oracle(gpu, c2, d):
    """The narrow widths the 1 x F column grids run at C2 size (d = 64 / F), through their default
    source-sliced schedules (4 / 8 / 12 MB slices: lgcn_amd.plan.slice_bytes_for): the K=3 forward
    per row within 1e-5 of the C oracle, and one layer bitwise on every unsplit row."""
    from lgcn_amd import propagate_forward
    from lgcn_amd.plan import slice_bytes_for
    from lgcn_amd.propagate import lgconv_forward

    g, plan = c2
    assert slice_bytes_for(g.num_nodes, d) > 0
    sched = plan.schedule("fwd", d)
    assert hasattr(sched, "launches")  # the sliced schedule, not the plain one
    rng = np.random.default_rng(d)
    uw = (rng.standard_normal((g.num_users, d)) * 0.01).astype(np.float32)
    iw = (rng.standard_normal((g.num_items, d)) * 0.01).astype(np.float32)
    out = propagate_forward(torch.from_numpy(uw).to(gpu), torch.from_numpy(iw).to(gpu), plan, 3).cpu().numpy()
    ru, ri = c_oracle.lightgcn_forward(uw, iw, g.edge_index, 3)
    assert_rows_close(out, np.concatenate([ru, ri]))
    x = np.concatenate([uw, iw])
    y = lgconv_forward(torch.from_numpy(x).to(gpu), plan).cpu().numpy()
    _, w = c_oracle.gcn_norm(g.edge_index, g.num_nodes)
    ref = c_oracle.lgconv(x, g.edge_index, w)
    mask = np.ones(g.num_nodes, bool)
    mask[sched.splits[: sched.n_splits, 0].cpu().numpy()] = False
    assert np.array_equal(y[mask], ref[mask])


def test_c2_single_layer_bitwise_on_unsplit_rows(gpu, c2):
    """One layer: every row summed as one sequential chain (not cut into chunks — with the
    source-sliced schedule, a chain that runs through several slice launches) is bitwise the
    reference CPU scatter_add_ result; split (hub) rows — up to 62k terms each — are within 1e-5
    relative and, against the exact float64 sums, no worse than the sequential CPU order: their
    root-mean-square error over every split-row entry is at most the sequential order's (the
    largest single-entry errors are printed next to each other)."""
    from lgcn_amd.propagate import lgconv_forward

    g, plan = c2
    x = (np.random.default_rng(2).standard_normal((g.num_nodes, 64)) * 0.01).astype(np.float32)
    y = lgconv_forward(torch.from_numpy(x).to(gpu), plan).cpu().numpy()
    _, w = c_oracle.gcn_norm(g.edge_index, g.num_nodes)
    ref = c_oracle.lgconv(x, g.edge_index, w)
    sched = plan.schedule("fwd", 64)  # the source-sliced schedule at this size (lgcn_amd.sliced)
    split_rows = sched.splits[: sched.n_splits, 0].cpu().numpy()
    mask = np.ones(g.num_nodes, bool)
    mask[split_rows] = False
    assert mask.sum() > 0.9 * g.num_nodes
    assert np.array_equal(y[mask], ref[mask])
    assert_rows_close(y[~mask], ref[~mask])
    # split rows: against the exact (float64) sum the chunked order is no worse than the
    # reference's sequential order
    src, dst = g.edge_index
    sel = ~mask[dst]
    pos = np.full(g.num_nodes, -1)
    pos[~mask] = np.arange((~mask).sum())
    rows = pos[dst[sel]]
    wx = w[sel].astype(np.float64)
    exact = np.stack([np.bincount(rows, weights=wx * x[src[sel], c], minlength=(~mask).sum()) for c in range(64)], 1)
    e_hip, e_ref = y[~mask] - exact, ref[~mask] - exact
    rms_hip, rms_ref = float(np.sqrt(np.mean(e_hip ** 2))), float(np.sqrt(np.mean(e_ref ** 2)))
    print(f"split rows vs exact: rms {rms_hip:.3g} (chunked) vs {rms_ref:.3g} (sequential); "
          f"max {np.abs(e_hip).max():.3g} vs {np.abs(e_ref).max():.3g}")
    assert rms_hip <= rms_ref, (rms_hip, rms_ref)


def test_c2_adjoint_and_linear(gpu, c2):
    """<Â x, y> == <x, Âᵀ y> (forward plan vs transposed plan) and Â(a x + b y) == a Âx + b Ây."""
    from lgcn_amd.propagate import lgconv_backward, lgconv_forward

    g, plan = c2
    N = g.num_nodes
    gen = torch.Generator(device=gpu).manual_seed(1)
    x = torch.randn(N, 64, device=gpu, generator=gen)
    y = torch.randn(N, 64, device=gpu, generator=gen)
    ax = lgconv_forward(x, plan)
    aty = lgconv_backward(y, plan)
    lhs = (ax.double() * y.double()).sum().item()
    rhs = (x.double() * aty.double()).sum().item()
    assert abs(lhs - rhs) <= 1e-5 * (ax.double().norm() * y.double().norm()).item()
    comb = lgconv_forward(2.0 * x - 3.0 * y, plan)
    expect = 2.0 * ax - 3.0 * lgconv_forward(y, plan)
    assert_rows_close(comb.cpu().numpy(), expect.cpu().numpy(), what="linearity")
