"""The harness mirror (package utils/train_test.py, utils/helpers.py) vs outputs of the
reference's own utils/train_test.py and utils/helpers.py (tests/golden/harness.npz, made by
tests/golden/make_golden.py). Everything here runs on CPU; equality is bitwise — on a host whose CPU
torch kernels round as the recording host's did (this container). On another host CPU (the GPU
box's) torch's vectorised CPU reductions may round differently and the post-epoch tables move at the
last bit; the GPU counterpart with tolerances is tests/test_gpu_harness.py::
test_harness_epoch_and_evaluate_match_reference_golden."""
import numpy as np
import torch

from conftest import GOLDEN
from oracle.lgconv_torch import OracleLightGCN
from utils import helpers as H
from utils import train_test as TT

G = np.load(GOLDEN / "harness.npz")


class _Batch:
    def __init__(self, ei):
        self.edge_index = ei

    def to(self, device):
        return self


def test_bpr_loss_matches_reference():
    ins = [torch.from_numpy(a.copy()).requires_grad_(True) for a in G["bpr_inputs"]]
    loss = TT.bpr_loss(*ins)
    loss.backward()
    assert np.float32(loss.item()) == G["bpr_loss"]
    for t, g in zip(ins, G["bpr_grads"]):
        assert np.array_equal(t.grad.numpy(), g)


def test_triplets_match_reference():
    torch.manual_seed(123)
    u, p, n = H.get_triplets_indices(torch.from_numpy(G["trip_edge_index"]), int(G["trip_U"]), int(G["trip_I"]),
                                     torch.device("cpu"))
    assert np.array_equal(u.numpy(), G["trip_users"])
    assert np.array_equal(p.numpy(), G["trip_pos"])
    assert np.array_equal(n.numpy(), G["trip_neg"])
    assert u.numel() == p.numel() == n.numel()


def test_recall_matches_reference():
    embs = tuple(torch.from_numpy(a.copy()) for a in G["recall_embs"])
    for k in (20, 100):
        np.random.seed(7)
        assert TT.compute_recall_at_k(embs, k=k) == float(G[f"recall_k{k}"])


def _trained_model():
    U, I = int(G["train_U"]), int(G["train_I"])
    model = OracleLightGCN(U, I, num_layers=3, dim_h=64)
    with torch.no_grad():
        model.user_embedding.weight.copy_(torch.from_numpy(G["train_init_user_w"]))
        model.item_embedding.weight.copy_(torch.from_numpy(G["train_init_item_w"]))
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    loader = [_Batch(torch.from_numpy(G[f"train_batch{p}"])) for p in range(3)]
    torch.manual_seed(41)
    loss = TT.train(model, opt, loader, torch.device("cpu"))
    return model, loss


def test_train_epoch_matches_reference():
    model, loss = _trained_model()
    assert loss == float(G["train_epoch_loss"])
    assert np.array_equal(model.user_embedding.weight.detach().numpy(), G["train_user_w"])
    assert np.array_equal(model.item_embedding.weight.detach().numpy(), G["train_item_w"])


def test_evaluate_matches_reference():
    model, _ = _trained_model()
    torch.manual_seed(42)
    np.random.seed(43)
    vloss, vrec = TT.evaluate(model, _Batch(torch.from_numpy(G["val_edge_index"])), torch.device("cpu"))
    assert vloss == float(G["val_loss"])
    assert vrec == float(G["val_recall100"])


def test_recall_upper_bound():
    """Q6: Recall@k under the reference definition is at most k / #positives."""
    rng = np.random.default_rng(0)
    embs = tuple(torch.from_numpy(rng.standard_normal((500, 8)).astype(np.float32)) for _ in range(3))
    np.random.seed(0)
    assert TT.compute_recall_at_k(embs, k=20) <= 20 / 500 + 1e-12


def test_train_routes_cpu_models_to_the_reference_loop():
    """The package's train() runs the fused batch step only for a HIP LightGCN with the reference's
    torch Adam (lgcn_amd.harness.eligibility); a CPU model takes the reference loop — bitwise the
    reference's results (test_train_epoch_matches_reference) — and the harness says why."""
    _trained_model()
    assert TT.LAST_TRAIN_PATH == "reference: model not on a ROCm device"


def test_fused_harness_eligibility_reasons():
    from lgcn_amd import harness

    model = OracleLightGCN(10, 8, num_layers=2, dim_h=16)
    assert "ROCm" in harness.eligibility(model, torch.optim.Adam(model.parameters(), lr=1e-3))

    class Bare(torch.nn.Module):
        pass

    assert "not a LightGCN" in harness.eligibility(Bare(), None)
