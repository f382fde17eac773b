"""The CPU oracle, pinned: numpy and C restatements vs the golden LGConv cases (PyG 2.4.0 op
sequence on torch CPU primitives, tests/golden/make_golden.py), bit for bit."""
import numpy as np
import pytest

from conftest import GOLDEN
from oracle import c_oracle
from oracle import lgconv_ref as R

_G = np.load(GOLDEN / "lgconv_cases.npz")
CASES = [str(c) for c in _G["cases"]]


def case(name):
    return {k.split("__", 1)[1]: _G[k] for k in _G.files if k.startswith(name + "__")}


@pytest.mark.parametrize("name", CASES)
def test_gcn_norm_matches_golden(name):
    c = case(name)
    N = int(c["U"] + c["I"])
    assert np.array_equal(R.gcn_norm(c["edge_index"], N), c["w"])
    _, w = c_oracle.gcn_norm(c["edge_index"], N)
    assert np.array_equal(w, c["w"])


@pytest.mark.parametrize("name", CASES)
def test_csr_order_matches_golden(name):
    """Stable grouping by target (forward) and by source (transposed) == torch.sort(stable)."""
    c = case(name)
    N = int(c["U"] + c["I"])
    ei = c["edge_index"]
    for key, other, perm in ((ei[1], ei[0], c["perm_by_dst"]), (ei[0], ei[1], c["perm_by_src"])):
        rp, col, eid = R.csr_by_key(key, other, N)
        assert np.array_equal(eid, perm)
        rp2, col2, eid2 = c_oracle.csr_build(key, other, N)
        assert np.array_equal(rp, rp2) and np.array_equal(col, col2) and np.array_equal(eid, eid2)
        assert np.array_equal(col, other[perm])
        assert rp[-1] == ei.shape[1] and np.all(np.diff(rp) >= 0)


@pytest.mark.parametrize("name", CASES)
def test_forward_matches_golden(name):
    c = case(name)
    K = int(c["K"])
    u, i = R.lightgcn_forward(c["user_w"], c["item_w"], c["edge_index"], K)
    assert np.array_equal(u, c["users_out"]) and np.array_equal(i, c["items_out"])
    u2, i2 = c_oracle.lightgcn_forward(c["user_w"], c["item_w"], c["edge_index"], K)
    assert np.array_equal(u2, c["users_out"]) and np.array_equal(i2, c["items_out"])


@pytest.mark.parametrize("name", CASES)
def test_backward_matches_golden(name):
    c = case(name)
    K, U = int(c["K"]), int(c["U"])
    gu, gi = R.lightgcn_backward(c["dF"], c["edge_index"], U, K)
    assert np.array_equal(gu, c["grad_user"]) and np.array_equal(gi, c["grad_item"])
    gu2, gi2 = c_oracle.lightgcn_backward(c["dF"], c["edge_index"], U, K)
    assert np.array_equal(gu2, c["grad_user"]) and np.array_equal(gi2, c["grad_item"])


def test_toy_graph_is_reference_smoke_graph():
    """models/light_gcn.py:68-73: 10 users, 15 items, edges [[0..19],[10..19,0..9]], K=4 default."""
    c = case("toy")
    assert int(c["U"]) == 10 and int(c["I"]) == 15 and int(c["K"]) == 4 and int(c["d"]) == 64
    assert c["edge_index"].tolist() == [list(range(20)), list(range(10, 20)) + list(range(10))]
    # nodes 20..24 (items 10..14) have no edges: their final row is x0 / (K+1)^2
    x0_items = c["item_w"][10:]
    assert np.array_equal(c["items_out"][10:], (x0_items / np.float32(5)) * np.float32(0.2))


def test_zero_in_degree_source_gets_zero_weight():
    """Q3: after a directed subsample, a node can keep out-edges but lose every in-edge; its
    out-edges then carry weight 0 (deg^-1/2 = inf -> 0)."""
    ei = np.array([[0, 1, 2], [2, 2, 0]])  # node 1: out-edge only
    w = R.gcn_norm(ei, 3)
    assert w[1] == 0.0 and w[0] > 0 and w[2] > 0


def test_to_undirected_coalesces():
    ei = np.array([[0, 0, 1, 3], [3, 3, 2, 0]])
    out = R.to_undirected(ei, 4)
    assert out.tolist() == [[0, 1, 2, 3], [3, 2, 1, 0]]


def test_torch_restatement_agrees():
    """oracle/lgconv_torch.py (the cpu_baseline path) is the same arithmetic."""
    import torch

    from oracle.lgconv_torch import OracleLightGCN

    c = case("sub_K3_d64")
    U, I = int(c["U"]), int(c["I"])
    m = OracleLightGCN(U, I, 3, 64)
    with torch.no_grad():
        m.user_embedding.weight.copy_(torch.from_numpy(c["user_w"]))
        m.item_embedding.weight.copy_(torch.from_numpy(c["item_w"]))
    u, i = m(torch.from_numpy(c["edge_index"]))
    assert np.array_equal(u.detach().numpy(), c["users_out"])
