"""The harness's train() (reference utils/train_test.py:66-103) both ways on the GPU: the
reference-style loop (autograd + torch Adam + clip_grad_norm_, LGCN_HARNESS_FUSED=0) and the fused
batch step it routes to by default (lgcn_amd.harness: HIP forward / BPR / backward, exact row-lazy
Adam, one hipGraph per batch). Same model init, same seed, so the same negatives: the epoch loss
within 1e-5, and after every epoch the tables and Adam moments within 1e-5 per row on the elements
whose Adam steps are well conditioned (_settled: every step's gradient above 1e-4 of its row's
largest, as test_gpu_configs.py's C3 bar, and the first moment not a near-cancellation of
earlier gradients; those elements are counted and printed), the second moments within 1e-5 per row everywhere, the
rows that move identical, the step counts equal.
Epoch 2 starts from the torch optimizer state epoch 1 wrote back (the paths can alternate)."""
import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


class _Batch:
    def __init__(self, ei):
        self.edge_index = ei

    def to(self, device):
        return _Batch(self.edge_index.to(device))


def _run(gpu, monkeypatch, fused, U, I, d, init, loader, epochs=2):
    from models.light_gcn import LightGCN
    from utils import train_test as TT

    monkeypatch.setenv("LGCN_HARNESS_FUSED", "1" if fused else "0")
    model = LightGCN(U, I, num_layers=3, dim_h=d).to(gpu)
    with torch.no_grad():
        model.user_embedding.weight.copy_(init[0])
        model.item_embedding.weight.copy_(init[1])
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    grads = []
    if not fused:  # record every step's (pre-clip) gradients: the settled-element mask
        inner = opt.step

        def step(*a, **k):
            grads.append([p.grad.detach().clone() for p in (model.user_embedding.weight, model.item_embedding.weight)])
            return inner(*a, **k)

        opt.step = step
    out = []
    torch.manual_seed(41)
    for _ in range(epochs):
        loss = TT.train(model, opt, loader, gpu)
        path = TT.LAST_TRAIN_PATH
        st = [opt.state[p] for p in (model.user_embedding.weight, model.item_embedding.weight)]
        out.append(dict(loss=loss, path=path,
                        w=[model.user_embedding.weight.detach().cpu().numpy().copy(),
                           model.item_embedding.weight.detach().cpu().numpy().copy()],
                        m=[s["exp_avg"].cpu().numpy().copy() for s in st],
                        v=[s["exp_avg_sq"].cpu().numpy().copy() for s in st],
                        step=[float(s["step"]) for s in st]))
    return out, grads


def _settled(grads, frac=0.05, g_floor=1e-4):
    """Per table, the elements whose Adam update is well conditioned in every step: the first
    moment m_s (the reference's clipped gradients, beta1 = 0.9) is at least `frac` of the same
    average taken over |g|. Where it is smaller, m is a near-cancellation of earlier steps'
    gradients and its relative error — hence the step's, hence the weight's — is the gradients'
    1e-6-level summation-order differences amplified by that factor; those elements are counted,
    not held to the bar. (One step: m = 0.1 g, every nonzero gradient element is settled.)"""
    m = [np.zeros(g.shape, np.float64) for g in grads[0]]
    a = [np.zeros(g.shape, np.float64) for g in grads[0]]
    ok = [np.ones(g.shape, bool) for g in grads[0]]
    for gs in grads:
        gn = [g.double().cpu().numpy() for g in gs]
        norm = np.sqrt(sum(float((g * g).sum()) for g in gn))
        c = min(1.0, 1.0 / (norm + 1e-6))
        for t, g in enumerate(gn):
            m[t] = 0.9 * m[t] + 0.1 * c * g
            a[t] = 0.9 * a[t] + 0.1 * c * np.abs(g)
            ok[t] &= np.abs(m[t]) >= frac * a[t]
            # and each step's gradient clear of the per-row gradient bar (1e-5 of the row's largest)
            # by g_floor / 1e-5, or exactly 0: the paths' gradients agree to ~1e-6 of the ROW's
            # scale, and Adam moves every element by about lr whatever its size, so a small
            # element's larger relative error reaches its weight whole
            ok[t] &= (g == 0) | (np.abs(g) > g_floor * np.abs(g).max(axis=1, keepdims=True))
    return ok


def _compare(ref, got, grads, w0, what):
    from parity import assert_rows_close

    n_steps = 0
    for e, (r, g) in enumerate(zip(ref, got)):
        assert r["path"].startswith("reference") and g["path"] == "fused", (r["path"], g["path"])
        assert abs(g["loss"] - r["loss"]) <= 1e-5 * abs(r["loss"]), (e, g["loss"], r["loss"])
        assert g["step"] == r["step"], (g["step"], r["step"])
        n_steps = int(r["step"][0])
        stats = {}
        masks = _settled(grads[:n_steps])
        for t, name in enumerate(("user", "item")):
            settled = masks[t]
            # the same rows move
            assert np.array_equal(np.any(g["w"][t] != w0[t], axis=1), np.any(r["w"][t] != w0[t], axis=1)), name
            for key in ("w", "m"):
                a, b = g[key][t], r[key][t]
                diff = np.where(settled, np.abs(a - b), 0.0)
                scale = np.abs(b).max(axis=1)
                worst = float((diff.max(axis=1) / np.where(scale > 0, scale, 1.0)).max())
                assert worst <= 1e-5, (what, e, name, key, worst)
                stats[f"{name}.{key}"] = worst
            # second moments: g^2 sums, no sign question — every row within 1e-5 of its scale
            assert_rows_close(g["v"][t], r["v"][t], rtol=1e-5, what=f"{what} epoch {e} {name} exp_avg_sq")
            stats[f"{name}.unsettled"] = int((~settled).sum())
        print(f"{what} epoch {e}: loss {g['loss']:.8f} vs {r['loss']:.8f}, steps {n_steps}, worst row-rel {stats}")


def test_harness_train_fused_matches_reference_loop_golden(gpu, monkeypatch):
    """The golden harness graph's three cluster batches (tests/golden/harness.npz, d = 64)."""
    G = np.load(GOLDEN / "harness.npz")
    U, I = int(G["train_U"]), int(G["train_I"])
    init = (torch.from_numpy(G["train_init_user_w"]), torch.from_numpy(G["train_init_item_w"]))
    loader = [_Batch(torch.from_numpy(G[f"train_batch{p}"])) for p in range(3)]
    ref, grads = _run(gpu, monkeypatch, False, U, I, 64, init, loader)
    got, _ = _run(gpu, monkeypatch, True, U, I, 64, init, loader)
    w0 = [init[0].numpy(), init[1].numpy()]
    _compare(ref, got, grads, w0, "golden")


def test_harness_train_fused_matches_reference_loop_c3(gpu, monkeypatch):
    """C3 batches (ML-25M-shaped graph, 1024 parts, 32 parts per batch, K=3, d=128). One step (a
    one-batch epoch): the loss within 1e-5, the tables and both moments per row within 1e-5 on the
    settled elements — test_gpu_configs.py's C3 bar. Four batches, two epochs: every epoch's loss
    within 1e-5; the tables' drift is printed, not asserted — after the first step the two paths
    take their gradients at weights that already differ where Adam's sign-like step met a
    noise-level gradient, and each later step carries that on (the same reason the lazy / dense
    optimizer comparison in test_gpu_training.py asserts one step and prints twenty)."""
    from lgcn_amd import cluster, synth

    g = synth.ml25m_shaped(seed=0)
    train = synth.train_split(g.edge_index, 0.9, seed=0)
    _, _, batches = cluster.cluster_batches(train, g.num_nodes, 1024, 32)
    U, I, d = g.num_users, g.num_items, 128
    torch.manual_seed(0)
    init = (torch.randn(U, d) * 0.01, torch.randn(I, d) * 0.01)
    w0 = [init[0].numpy(), init[1].numpy()]
    one = [_Batch(torch.from_numpy(batches[0]))]
    ref, grads = _run(gpu, monkeypatch, False, U, I, d, init, one, epochs=1)
    got, _ = _run(gpu, monkeypatch, True, U, I, d, init, one, epochs=1)
    _compare(ref, got, grads, w0, "C3 one step")
    four = [_Batch(torch.from_numpy(b)) for b in batches[:4]]
    ref, _ = _run(gpu, monkeypatch, False, U, I, d, init, four, epochs=2)
    got, _ = _run(gpu, monkeypatch, True, U, I, d, init, four, epochs=2)
    for e, (r, q) in enumerate(zip(ref, got)):
        assert q["path"] == "fused" and r["path"].startswith("reference")
        assert abs(q["loss"] - r["loss"]) <= 1e-5 * abs(r["loss"]), (e, q["loss"], r["loss"])
        assert q["step"] == r["step"]
        drift = max(float(np.abs(q["w"][t] - r["w"][t]).max()) for t in range(2))
        print(f"C3 4 batches, epoch {e}: loss {q['loss']:.8f} vs {r['loss']:.8f}; max |w| difference {drift:.3g}")


def test_harness_train_falls_back(gpu, monkeypatch):
    """What the fused step does not reproduce runs the reference loop (and says why)."""
    from models.light_gcn import LightGCN
    from utils import train_test as TT

    G = np.load(GOLDEN / "harness.npz")
    U, I = int(G["train_U"]), int(G["train_I"])
    loader = [_Batch(torch.from_numpy(G[f"train_batch{p}"])) for p in range(3)]
    model = LightGCN(U, I, num_layers=3, dim_h=64).to(gpu)
    TT.train(model, torch.optim.SGD(model.parameters(), lr=1e-3), loader, gpu)
    assert TT.LAST_TRAIN_PATH.startswith("reference") and "SGD" in TT.LAST_TRAIN_PATH
    TT.train(model, torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-4), loader, gpu)
    assert TT.LAST_TRAIN_PATH.startswith("reference")
    bad = [_Batch(torch.tensor([[0, U], [1, U + 1]]))]  # a user-user and an item-item edge: not bipartite
    TT.train(model, torch.optim.Adam(model.parameters(), lr=1e-3), bad, gpu)
    assert TT.LAST_TRAIN_PATH.startswith("reference") and "bipartite" in TT.LAST_TRAIN_PATH
