"""Every golden case (tests/golden/lgconv_cases.npz: outputs of the reference's OWN LightGCN
class, reference models/light_gcn.py:13-40, with PyG 2.4.0's LGConv restated on torch CPU
primitives; see tests/golden/make_golden.py) run through the HIP path on the GPU.

* Through the drop-in class (models.light_gcn.LightGCN, default plan): forward outputs and both
  weight gradients within 1e-5 per row (tests/parity.py).
* Through the propagation entry points with every row one schedule item (chunk >= max degree):
  forward and backward BIT-IDENTICAL to the reference class.
* The plan's CSR order and gcn_norm weights are bitwise the golden ones.
"""
import numpy as np
import pytest
import torch

from conftest import GOLDEN
from parity import assert_rows_close

pytestmark = pytest.mark.gpu

_G = np.load(GOLDEN / "lgconv_cases.npz")
CASES = [str(c) for c in _G["cases"]]


def case(name):
    return {k.split("__", 1)[1]: _G[k] for k in _G.files if k.startswith(name + "__")}


@pytest.mark.parametrize("name", CASES)
def test_golden_through_lightgcn_class(gpu, name):
    from models.light_gcn import LightGCN

    c = case(name)
    U, I, K, d = (int(c[k]) for k in ("U", "I", "K", "d"))
    model = LightGCN(U, I, num_layers=K, dim_h=d).to(gpu)
    with torch.no_grad():
        model.user_embedding.weight.copy_(torch.from_numpy(c["user_w"]))
        model.item_embedding.weight.copy_(torch.from_numpy(c["item_w"]))
    users, items = model(torch.from_numpy(c["edge_index"]).to(gpu))
    rr_u, el_u = assert_rows_close(users.detach().cpu().numpy(), c["users_out"], what=f"{name} users")
    rr_i, el_i = assert_rows_close(items.detach().cpu().numpy(), c["items_out"], what=f"{name} items")
    (torch.cat([users, items]) * torch.from_numpy(c["dF"]).to(gpu)).sum().backward()
    rr_gu, _ = assert_rows_close(model.user_embedding.weight.grad.cpu().numpy(), c["grad_user"], what=f"{name} dU")
    rr_gi, _ = assert_rows_close(model.item_embedding.weight.grad.cpu().numpy(), c["grad_item"], what=f"{name} dI")
    print(f"{name}: row-rel fwd {max(rr_u, rr_i):.2e} (elementwise {max(el_u, el_i):.2e}), "
          f"bwd {max(rr_gu, rr_gi):.2e}")


@pytest.mark.parametrize("name", CASES)
def test_golden_bitwise_unsplit(gpu, name):
    from lgcn_amd import propagate_backward, propagate_forward
    from lgcn_amd.plan import PropagationPlan

    c = case(name)
    U, I, K, d = (int(c[k]) for k in ("U", "I", "K", "d"))
    N = U + I
    ei = torch.from_numpy(c["edge_index"]).to(gpu)
    plan = PropagationPlan(ei, N, chunk=1 << 20)
    assert plan.fwd.n_splits == 0
    assert np.array_equal(plan.fwd.eid.cpu().numpy(), c["perm_by_dst"])
    assert np.array_equal(plan.bwd.eid.cpu().numpy(), c["perm_by_src"])
    assert np.array_equal(plan.fwd.val.cpu().numpy(), c["w"][c["perm_by_dst"]])
    out = propagate_forward(torch.from_numpy(c["user_w"]).to(gpu), torch.from_numpy(c["item_w"]).to(gpu), plan, K)
    out = out.cpu().numpy()
    assert np.array_equal(out[:U], c["users_out"]) and np.array_equal(out[U:], c["items_out"])
    gu, gi = propagate_backward(torch.from_numpy(c["dF"]).to(gpu), plan, U, K)
    assert np.array_equal(gu.cpu().numpy(), c["grad_user"]) and np.array_equal(gi.cpu().numpy(), c["grad_item"])
