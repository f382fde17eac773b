"""The harness's train() (reference utils/train_test.py:66-103) both ways on the GPU: the
reference-style loop (autograd + torch Adam + clip_grad_norm_, tuning harness_fused=False) and the fused
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


# the share of moved elements outside the 1e-5 row bar after 4-8 steps of the C3 batches: at most
# 1.1e-4 in the captured runs (profiles/r05d_parity/: 282 of 2.6M user elements after 8 steps,
# max |dw| 9.7e-6 against the 2 lr steps = 1.6e-2 allowed) — bound 1e-3, ~9x
MULTI_STEP_OFF_BAR_FRAC = 1e-3


class _Batch:
    def __init__(self, ei):
        self.edge_index = ei

    def to(self, device):
        return _Batch(self.edge_index.to(device))


def _run(gpu, tune, fused, U, I, d, init, loader, epochs=2):
    from models.light_gcn import LightGCN
    from utils import train_test as TT

    tune(harness_fused=bool(fused))
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


def _compare(ref, got, grads, w0, what, lr=1e-3):
    from parity import assert_rows_close, record_stats, trajectory_bar

    n_steps = 0
    for e, (r, g) in enumerate(zip(ref, got)):
        assert r["path"].startswith("reference") and g["path"] == "fused", (r["path"], g["path"])
        assert abs(g["loss"] - r["loss"]) <= 1e-5 * abs(r["loss"]), (e, g["loss"], r["loss"])
        assert g["step"] == r["step"], (g["step"], r["step"])
        n_steps = int(r["step"][0])
        stats = {"loss": g["loss"], "loss_ref": r["loss"]}
        masks = _settled(grads[:n_steps])
        for t, name in enumerate(("user", "item")):
            settled = masks[t]
            # the same rows move
            assert np.array_equal(np.any(g["w"][t] != w0[t], axis=1), np.any(r["w"][t] != w0[t], axis=1)), name
            # weights: settled elements within 1e-5 of their row's scale, every element within
            # 2 lr per step, the unsettled share of the moved elements bounded (tests/parity.py)
            stats[f"{name}.w"] = trajectory_bar(g["w"][t], r["w"][t], w0[t], settled, lr, n_steps,
                                                f"{what} epoch {e} {name} weights")
            a, b = g["m"][t], r["m"][t]
            diff = np.where(settled, np.abs(a - b), 0.0)
            scale = np.abs(b).max(axis=1)
            worst = float((diff.max(axis=1) / np.where(scale > 0, scale, 1.0)).max())
            assert worst <= 1e-5, (what, e, name, "m", worst)
            stats[f"{name}.m_settled_row_rel"] = worst
            # second moments: g^2 sums, no sign question — every row within 1e-5 of its scale
            stats[f"{name}.v_row_rel"] = assert_rows_close(g["v"][t], r["v"][t], rtol=1e-5,
                                                           what=f"{what} epoch {e} {name} exp_avg_sq")[0]
        record_stats(f"harness_{what.replace(' ', '_')}_epoch{e}", stats)
        print(f"{what} epoch {e}: loss {g['loss']:.8f} vs {r['loss']:.8f}, steps {n_steps}, {stats}")


def test_harness_train_fused_matches_reference_loop_golden(gpu, tune):
    """The golden harness graph's three cluster batches (tests/golden/harness.npz, d = 64)."""
    G = np.load(GOLDEN / "harness.npz")
    U, I = int(G["train_U"]), int(G["train_I"])
    init = (torch.from_numpy(G["train_init_user_w"]), torch.from_numpy(G["train_init_item_w"]))
    loader = [_Batch(torch.from_numpy(G[f"train_batch{p}"])) for p in range(3)]
    ref, grads = _run(gpu, tune, False, U, I, 64, init, loader)
    got, _ = _run(gpu, tune, True, U, I, 64, init, loader)
    w0 = [init[0].numpy(), init[1].numpy()]
    _compare(ref, got, grads, w0, "golden")


def test_harness_train_fused_matches_reference_loop_c3(gpu, tune):
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
    ref, grads = _run(gpu, tune, False, U, I, d, init, one, epochs=1)
    got, _ = _run(gpu, tune, True, U, I, d, init, one, epochs=1)
    _compare(ref, got, grads, w0, "C3 one step")
    four = [_Batch(torch.from_numpy(b)) for b in batches[:4]]
    ref, _ = _run(gpu, tune, False, U, I, d, init, four, epochs=2)
    got, _ = _run(gpu, tune, True, U, I, d, init, four, epochs=2)
    from parity import record_stats, trajectory_bar

    for e, (r, q) in enumerate(zip(ref, got)):
        assert q["path"] == "fused" and r["path"].startswith("reference")
        assert abs(q["loss"] - r["loss"]) <= 1e-5 * abs(r["loss"]), (e, q["loss"], r["loss"])
        assert q["step"] == r["step"]
        steps = int(r["step"][0])
        stats = {"loss": q["loss"], "loss_ref": r["loss"]}
        for t, name in enumerate(("user", "item")):
            # after the first step the paths take gradients at weights that already differ where
            # Adam's sign-like step met a noise-level gradient: here "settled" is simply the
            # elements inside the 1e-5 row bar, and the share outside it is what is bounded
            a, b = q["w"][t].astype(np.float64), r["w"][t].astype(np.float64)
            scale = np.abs(b).max(axis=1, keepdims=True)
            inside = np.abs(a - b) <= 1e-5 * np.where(scale > 0, scale, 1.0)
            stats[f"{name}.w"] = trajectory_bar(q["w"][t], r["w"][t], w0[t], inside, 1e-3, steps,
                                                f"C3 4 batches epoch {e} {name}", max_frac=MULTI_STEP_OFF_BAR_FRAC)
        record_stats(f"harness_C3_4batches_epoch{e}", stats)
        print(f"C3 4 batches, epoch {e}: loss {q['loss']:.8f} vs {r['loss']:.8f}; {stats}")


def test_harness_train_falls_back(gpu, tune):
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


class _FreshLoader:
    """Collates a new edge_index tensor on every iteration, as the reference's PyG
    DataLoader(batch_size=1, shuffle=True) does (reference data/dataset_handler.py:285)."""

    def __init__(self, arrays):
        self.arrays = arrays

    def __len__(self):
        return len(self.arrays)

    def __iter__(self):
        for a in self.arrays:
            yield _Batch(torch.from_numpy(a.copy()))


def _epochs(gpu, U, I, init, loader, epochs):
    from lgcn_amd import harness
    from models.light_gcn import LightGCN
    from utils import train_test as TT

    model = LightGCN(U, I, num_layers=3, dim_h=64).to(gpu)
    with torch.no_grad():
        model.user_embedding.weight.copy_(init[0])
        model.item_embedding.weight.copy_(init[1])
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    torch.manual_seed(41)
    losses, mem = [], []
    for _ in range(epochs):
        losses.append(TT.train(model, opt, loader, gpu))
        assert TT.LAST_TRAIN_PATH == "fused", TT.LAST_TRAIN_PATH
        torch.cuda.synchronize()
        mem.append(torch.cuda.memory_allocated(gpu))
    w = [model.user_embedding.weight.detach().cpu().clone(), model.item_embedding.weight.detach().cpu().clone()]
    return losses, w, harness._FAST[opt], mem


def test_harness_fresh_tensors_each_epoch_replay(gpu, tune):
    """a loader that collates new edge_index tensors every epoch finds each
    batch's state (plans, captured hipGraph) by content — bitwise the same run as a loader that
    yields the same objects, one state per distinct batch, no memory growth across epochs."""
    tune(harness_fused=True)
    G = np.load(GOLDEN / "harness.npz")
    U, I = int(G["train_U"]), int(G["train_I"])
    init = (torch.from_numpy(G["train_init_user_w"]), torch.from_numpy(G["train_init_item_w"]))
    arrays = [G[f"train_batch{p}"] for p in range(3)]
    same = [_Batch(torch.from_numpy(a)) for a in arrays]
    l_same, w_same, _, _ = _epochs(gpu, U, I, init, same, 4)
    l_fresh, w_fresh, fast, mem = _epochs(gpu, U, I, init, _FreshLoader(arrays), 4)
    assert l_same == l_fresh, (l_same, l_fresh)
    for a, b in zip(w_same, w_fresh):
        assert torch.equal(a, b)
    states = fast.step._states
    assert len(states) == 3, len(states)
    assert states.misses == 3 and states.hits_content + states.hits_object >= 9, \
        (states.misses, states.hits_content, states.hits_object)
    assert all(getattr(st, "graph", None) is not None for st in states.values())  # captured, replayed
    assert mem[1] == mem[2] == mem[3], mem


def test_harness_reg_rows_in_update_bitwise(gpu, tune):
    """ABI 10: the harness step with the BPR reg rows formed in the clip norm and the update, and its
    epoch-loss sum riding in the fused loss's workgroup (lgcn_range_scatter_add_counts), is bitwise
    the step with the two reg passes and its own lgcn_loss_accumulate launch: epoch losses and
    tables over 3 epochs of the golden batches."""
    tune(harness_fused=True)
    G = np.load(GOLDEN / "harness.npz")
    U, I = int(G["train_U"]), int(G["train_I"])
    init = (torch.from_numpy(G["train_init_user_w"]), torch.from_numpy(G["train_init_item_w"]))
    same = [_Batch(torch.from_numpy(G[f"train_batch{p}"])) for p in range(3)]
    out = {}
    for flag in (False, True):
        tune(reg_in_update=flag)
        losses, w, fast, _ = _epochs(gpu, U, I, init, same, 3)
        assert fast.step.reg_in_update == flag
        out[flag] = (losses, w)
    assert out[False][0] == out[True][0], out
    for a, b in zip(out[False][1], out[True][1]):
        assert torch.equal(a, b)


def test_harness_one_shot_loader_falls_back_mid_epoch(gpu, tune):
    """a non-bipartite batch after fused steps hands the rest of the epoch to the
    reference loop — the fused steps' Adam state written back first, no batch lost from a one-shot
    iterator (4 batches -> 4 Adam steps in the torch optimizer)."""
    from models.light_gcn import LightGCN
    from utils import train_test as TT

    tune(harness_fused=True)
    G = np.load(GOLDEN / "harness.npz")
    U, I = int(G["train_U"]), int(G["train_I"])
    good = [_Batch(torch.from_numpy(G[f"train_batch{p}"])) for p in range(3)]
    bad = _Batch(torch.tensor([[0, U], [1, U + 1]]))
    model = LightGCN(U, I, num_layers=3, dim_h=64).to(gpu)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    loss = TT.train(model, opt, iter([good[0], good[1], bad, good[2]]), gpu)
    assert np.isfinite(loss)
    assert TT.LAST_TRAIN_PATH.startswith("reference: fused for 2 batch(es)"), TT.LAST_TRAIN_PATH
    for p in (model.user_embedding.weight, model.item_embedding.weight):
        assert int(float(opt.state[p]["step"])) == 4
    # the next epoch starts fused again from the written-back state
    TT.train(model, opt, good, gpu)
    assert TT.LAST_TRAIN_PATH == "fused"
    for p in (model.user_embedding.weight, model.item_embedding.weight):
        assert int(float(opt.state[p]["step"])) == 7


def test_harness_epoch_and_evaluate_match_reference_golden(gpu, tune, monkeypatch):
    """the reference's own train() epoch and evaluate() outputs
    (tests/golden/harness.npz, recorded by running reference utils/train_test.py on the CPU oracle
    model: torch.manual_seed(41) -> train over the three golden batches, then torch.manual_seed(42),
    np.random.seed(43) -> evaluate on the validation edges) reproduced by this package's fused GPU
    train() and GPU evaluate(). The negatives are the reference's draws: the CPU global generator,
    moved to the device. Bars: the epoch loss and the validation loss within 1e-5 relative; the
    tables under the trajectory bar (settled elements — every step's gradient clear of the row bar
    in the reference run, no near-cancelling first moment — within 1e-5 of their row's scale);
    Recall@100's hit counts exact with recall_ties="cpu" (CPU torch.topk's choice among equal scores: the
    golden ran on a CPU), and with the default "index" rule equal to the oracle tables scored through
    that same rule."""
    from models.light_gcn import LightGCN
    from oracle.lgconv_torch import OracleLightGCN
    from parity import record_stats, trajectory_bar
    from utils import helpers
    from utils import train_test as TT

    monkeypatch.setattr(helpers, "sample_negative",
                        lambda pos_idx, num_items, device: torch.randint(0, num_items, (pos_idx.shape[0],)).to(device))
    G = np.load(GOLDEN / "harness.npz")
    U, I = int(G["train_U"]), int(G["train_I"])
    w0 = [G["train_init_user_w"], G["train_init_item_w"]]
    loader = [_Batch(torch.from_numpy(G[f"train_batch{p}"])) for p in range(3)]
    val = _Batch(torch.from_numpy(G["val_edge_index"]))

    def make(cls, dev):
        m = cls(U, I, num_layers=3, dim_h=64).to(dev)
        with torch.no_grad():
            m.user_embedding.weight.copy_(torch.from_numpy(w0[0]))
            m.item_embedding.weight.copy_(torch.from_numpy(w0[1]))
        return m

    # the reference run's per-step gradients (CPU oracle) for the settled-element mask. Its tables
    # equal the golden's bitwise on the host that recorded it (tests/test_harness.py); on another
    # host CPU torch's vectorised reductions may round differently, so they are not asserted here
    ref = make(OracleLightGCN, torch.device("cpu"))
    ropt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    grads, inner = [], ropt.step

    def step(*a, **k):
        grads.append([p.grad.detach().clone() for p in (ref.user_embedding.weight, ref.item_embedding.weight)])
        return inner(*a, **k)

    ropt.step = step
    torch.manual_seed(41)
    TT.train(ref, ropt, loader, torch.device("cpu"))

    tune(harness_fused=True)
    hip = make(LightGCN, gpu)
    opt = torch.optim.Adam(hip.parameters(), lr=1e-3)
    torch.manual_seed(41)
    loss = TT.train(hip, opt, loader, gpu)
    assert TT.LAST_TRAIN_PATH == "fused", TT.LAST_TRAIN_PATH
    gl = float(G["train_epoch_loss"])
    assert abs(loss - gl) <= 1e-5 * abs(gl), (loss, gl)
    masks = _settled(grads)
    stats = {"epoch_loss": loss, "epoch_loss_golden": gl}
    for t, (name, key) in enumerate((("user", "train_user_w"), ("item", "train_item_w"))):
        got = getattr(hip, f"{name}_embedding").weight.detach().cpu().numpy()
        stats[f"{name}.w"] = trajectory_bar(got, G[key], w0[t], masks[t], 1e-3, len(grads), f"golden epoch {name}")
    out = {}
    for ties in ("cpu", "index"):
        tune(recall_ties=ties)
        torch.manual_seed(42)
        np.random.seed(43)
        out[ties] = TT.evaluate(hip, val, gpu)
    # the oracle tables through the "index" rule on the GPU (the same negatives and picks)
    golden_model = _loaded(LightGCN, U, I, G, gpu)  # built before seeding: its init draws from the generator
    torch.manual_seed(42)
    np.random.seed(43)
    oracle_index = TT.evaluate(golden_model, val, gpu)
    vl, vr = float(G["val_loss"]), float(G["val_recall100"])
    stats.update(val_loss=out["cpu"][0], val_loss_golden=vl, recall100_cpu_ties=out["cpu"][1],
                 recall100_golden=vr, recall100_index=out["index"][1], recall100_index_oracle_tables=oracle_index[1])
    record_stats("harness_golden_epoch_evaluate", stats)
    print(f"golden epoch: loss {loss:.9f} vs {gl:.9f}; val loss {out['cpu'][0]:.9f} vs {vl:.9f}; Recall@100 "
          f"cpu ties {out['cpu'][1]:.9f} vs golden {vr:.9f}; index ties {out['index'][1]:.9f} "
          f"(oracle tables {oracle_index[1]:.9f}); {stats}")
    for ties in ("cpu", "index"):
        assert abs(out[ties][0] - vl) <= 1e-5 * abs(vl), (ties, out[ties][0], vl)
    # hit counts exact: one hit moves Recall@100 by 1 / (P * 100 * 10) — 1e-5 relative here — and
    # the 1e-9 left is the host CPU's float32 mean of 100 per-user values (another host, another
    # vector width)
    assert out["cpu"][1] == pytest.approx(vr, rel=1e-7, abs=0), (out["cpu"][1], vr)
    assert out["index"][1] == oracle_index[1], (out["index"][1], oracle_index[1])


def _loaded(cls, U, I, G, dev):
    """A model holding the golden post-epoch tables (the reference's own)."""
    m = cls(U, I, num_layers=3, dim_h=64).to(dev)
    with torch.no_grad():
        m.user_embedding.weight.copy_(torch.from_numpy(G["train_user_w"]))
        m.item_embedding.weight.copy_(torch.from_numpy(G["train_item_w"]))
    return m
