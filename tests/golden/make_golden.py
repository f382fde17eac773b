"""Generate the golden fixtures under tests/golden/ (run in the build container, where the
reference is mounted at /root/reference; the GPU box never runs this).

Two anchors, because the reference's hot path is split across two places:

1. harness.npz — the reference's OWN code, imported unmodified from /root/reference/utils
   (utils/train_test.py, utils/helpers.py; both import only torch/numpy/tqdm):
   bpr_loss (+ autograd grads), get_triplets_indices under a fixed torch seed,
   compute_recall_at_k under a fixed numpy seed, one train() epoch over three cluster batches
   with Adam(1e-3) + clip(1) (post-step weights), and evaluate() (loss, Recall@100).
   The model those harness functions drive is the reference's own LightGCN class (below).

2. lgconv_cases.npz — forward/backward of the reference's OWN LightGCN class: reference
   models/light_gcn.py:13-40 is loaded unmodified from /root/reference with its one missing
   import, ``torch_geometric.nn.LGConv`` (PyG 2.4.0, absent here: an ordinary
   ModuleNotFoundError), supplied IN MEMORY by oracle/lgconv_torch.py::OracleLGConv
   — PyG 2.4.0's LGConv op sequence (gcn_norm: scatter_add_ of ones, pow_(-0.5), masked_fill_;
   propagate: index_select, mul, scatter_add_) on torch CPU primitives. So the layer-stack mean
   (Q1), cat/split, the import-time seed and the N(0, 0.01) init are the reference's own code;
   only the LGConv arithmetic is a restatement (of a named third-party algorithm). Cases: the
   reference's own toy graph (models/light_gcn.py:68-73, seed-0 init, K=4 default) and seeded
   reference-shaped graphs: symmetric, 90 % directed subsample (Q3), shuffled union,
   hub-skewed, isolated nodes, and the C1 config (K=2, d=64, 50k edges). Gradients by autograd.
   CSR anchors: torch.sort(stable=True) order of edges by target and by source.

Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import pathlib
import sys

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
ROOT = HERE.parent.parent
REF = pathlib.Path("/root/reference")
sys.path.insert(0, str(ROOT / "movie-recommender-system-with-gnns_amd"))
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


# sha256 of each reference file this script executes, pinned when the fixtures were made: the
# reference tree is untrusted public content, so a file that changed is refused before it runs
REF_SHA256 = {
    "models/light_gcn.py": "a3177a4bc97a3bb9447a927717d0bf787b73bfc6f578df020a066e02fd1ff9a1",
    "utils/train_test.py": "6d0a86e09aff1ddbc25d8f68780cf80eec754a46882cc4aaea63d115f750cd7d",
    "utils/helpers.py": "986c99169ec54697227dd818421c8620e9cb16385b4aa0b98f006b06ed29dcba",
}


def check_reference_files() -> None:
    import hashlib

    for rel, want in REF_SHA256.items():
        got = hashlib.sha256((REF / rel).read_bytes()).hexdigest()
        if got != want:
            raise SystemExit(f"/root/reference/{rel} changed (sha256 {got}); refusing to execute it")


class Batch:
    """What the reference's train()/evaluate() need from a batch: .edge_index and .to()."""

    def __init__(self, edge_index):
        self.edge_index = edge_index

    def to(self, device):
        return self


def reference_lightgcn():
    """The reference's LightGCN class (models/light_gcn.py), loaded from /root/reference without
    modification. Its ``from torch_geometric.nn import LGConv`` is served by an in-memory module
    holding OracleLGConv; nothing is written anywhere (no bytecode, no files)."""
    import importlib.util
    import types

    from oracle.lgconv_torch import OracleLGConv

    if not REF.exists():
        raise SystemExit("/root/reference is not mounted: fixtures can only be made in the build container")
    check_reference_files()
    saved = {k: sys.modules.get(k) for k in ("torch_geometric", "torch_geometric.nn")}
    pyg = types.ModuleType("torch_geometric")
    pyg_nn = types.ModuleType("torch_geometric.nn")
    pyg_nn.LGConv = OracleLGConv
    pyg.nn = pyg_nn
    sys.modules["torch_geometric"], sys.modules["torch_geometric.nn"] = pyg, pyg_nn
    try:
        spec = importlib.util.spec_from_file_location("ref_light_gcn", REF / "models" / "light_gcn.py")
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    return mod.LightGCN


def lgconv_cases():
    import torch

    import graphs
    from lgcn_amd import synth
    from oracle.lgconv_torch import gcn_norm_torch

    RefLightGCN = reference_lightgcn()

    cases = {}

    def run(name, U, I, ei, K, d, weights=None, seed=0):
        torch.manual_seed(0)
        m = RefLightGCN(U, I, num_layers=K, dim_h=d)
        if weights is not None:
            with torch.no_grad():
                m.user_embedding.weight.copy_(torch.from_numpy(weights[0]))
                m.item_embedding.weight.copy_(torch.from_numpy(weights[1]))
        et = torch.from_numpy(np.ascontiguousarray(ei))
        u, i = m(et)
        dF = torch.from_numpy(np.random.default_rng(seed + 99).standard_normal((U + I, d)).astype(np.float32))
        (torch.cat([u, i]) * dF).sum().backward()
        w = gcn_norm_torch(et, U + I)
        by_dst = torch.sort(et[1], stable=True).indices
        by_src = torch.sort(et[0], stable=True).indices
        cases[name] = dict(
            U=np.int64(U), I=np.int64(I), K=np.int64(K), d=np.int64(d), edge_index=ei.astype(np.int64),
            user_w=m.user_embedding.weight.detach().numpy().copy(),
            item_w=m.item_embedding.weight.detach().numpy().copy(),
            users_out=u.detach().numpy(), items_out=i.detach().numpy(), dF=dF.numpy(),
            grad_user=m.user_embedding.weight.grad.numpy(), grad_item=m.item_embedding.weight.grad.numpy(),
            w=w.numpy(), perm_by_dst=by_dst.numpy().astype(np.int32), perm_by_src=by_src.numpy().astype(np.int32))

    # the reference's own smoke graph and defaults (num_layers=4, dim_h=64), seed-0 init
    U, I, ei = graphs.toy()
    run("toy", U, I, ei, 4, 64)
    run("sym_K3_d64", *graphs.sym(), 3, 64, weights=graphs.embeddings(300, 200, 64, 1), seed=1)
    run("sub_K3_d64", *graphs.subsampled(), 3, 64, weights=graphs.embeddings(300, 200, 64, 2), seed=2)
    U, I, ei = graphs.shuffled()
    run("shuf_K2_d8", U, I, ei, 2, 8, weights=graphs.embeddings(U, I, 8, 3), seed=3)
    U, I, ei = graphs.hub()
    run("hub_K3_d64", U, I, ei, 3, 64, weights=graphs.embeddings(U, I, 64, 4), seed=4)
    U, I, ei = graphs.with_isolated()
    run("iso_K1_d16", U, I, ei, 1, 16, weights=graphs.embeddings(U, I, 16, 5), seed=5)
    g = synth.bipartite(1000, 600, 25_000, seed=11)
    run("c1_K2_d64", g.num_users, g.num_items, g.edge_index, 2, 64,
        weights=graphs.embeddings(g.num_users, g.num_items, 64, 6), seed=6)
    flat = {f"{c}__{k}": v for c, arrs in cases.items() for k, v in arrs.items()}
    np.savez_compressed(HERE / "lgconv_cases.npz", cases=np.array(sorted(cases)), **flat)
    print("lgconv_cases:", sorted(cases))


def harness():
    import torch

    if not REF.exists():
        raise SystemExit("/root/reference is not mounted: harness fixtures can only be made in the build container")
    check_reference_files()
    sys.path.insert(0, str(REF / "utils"))
    import helpers as ref_helpers  # reference utils/helpers.py
    import train_test as ref_tt  # reference utils/train_test.py

    import graphs

    RefLightGCN = reference_lightgcn()
    out = {}
    # --- bpr_loss + grads
    rng = np.random.default_rng(21)
    B, d = 37, 16
    ins = [torch.from_numpy(rng.standard_normal((B, d)).astype(np.float32) * 0.1).requires_grad_(True)
           for _ in range(6)]
    loss = ref_tt.bpr_loss(*ins)
    loss.backward()
    out["bpr_inputs"] = np.stack([t.detach().numpy() for t in ins])
    out["bpr_loss"] = np.float32(loss.item())
    out["bpr_grads"] = np.stack([t.grad.numpy() for t in ins])
    # --- triplets
    U, I, ei = graphs.subsampled()
    et = torch.from_numpy(ei)
    torch.manual_seed(123)
    tu, tp, tn = ref_helpers.get_triplets_indices(et, U, I, torch.device("cpu"))
    out["trip_edge_index"] = ei
    out["trip_U"], out["trip_I"] = np.int64(U), np.int64(I)
    out["trip_users"], out["trip_pos"], out["trip_neg"] = tu.numpy(), tp.numpy(), tn.numpy()
    # --- recall@k
    rng = np.random.default_rng(22)
    Bv = 700
    r_embs = [torch.from_numpy(rng.standard_normal((Bv, 32)).astype(np.float32)) for _ in range(3)]
    out["recall_embs"] = np.stack([t.numpy() for t in r_embs])
    for k in (20, 100):
        np.random.seed(7)
        out[f"recall_k{k}"] = np.float64(ref_tt.compute_recall_at_k(tuple(r_embs), k=k))
    # --- one train() epoch over 3 cluster batches + evaluate(), reference harness end to end
    U, I, ei = graphs.sym(seed=31)
    rng = np.random.default_rng(32)
    perm = rng.permutation(ei.shape[1])
    n_val = ei.shape[1] // 10
    val_idx = np.sort(perm[:n_val])
    train_idx = np.sort(perm[n_val:])
    train_ei = ei[:, train_idx]
    part = rng.integers(0, 3, U + I)  # 3 'clusters': intra-part train edges, in train order
    batches = []
    for p in range(3):
        m = (part[train_ei[0]] == p) & (part[train_ei[1]] == p)
        batches.append(np.ascontiguousarray(train_ei[:, m]))
    torch.manual_seed(0)
    model = RefLightGCN(U, I, num_layers=3, dim_h=64)
    out["train_init_user_w"] = model.user_embedding.weight.detach().numpy().copy()
    out["train_init_item_w"] = model.item_embedding.weight.detach().numpy().copy()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    loader = [Batch(torch.from_numpy(b)) for b in batches]
    torch.manual_seed(41)
    epoch_loss = ref_tt.train(model, opt, loader, torch.device("cpu"))
    out["train_U"], out["train_I"] = np.int64(U), np.int64(I)
    for p, b in enumerate(batches):
        out[f"train_batch{p}"] = b
    out["train_epoch_loss"] = np.float64(epoch_loss)
    out["train_user_w"] = model.user_embedding.weight.detach().numpy().copy()
    out["train_item_w"] = model.item_embedding.weight.detach().numpy().copy()
    out["val_edge_index"] = np.ascontiguousarray(ei[:, val_idx])
    torch.manual_seed(42)
    np.random.seed(43)
    vloss, vrec = ref_tt.evaluate(model, Batch(torch.from_numpy(out["val_edge_index"])), torch.device("cpu"))
    out["val_loss"] = np.float64(vloss)
    out["val_recall100"] = np.float64(vrec)
    np.savez_compressed(HERE / "harness.npz", **out)
    print("harness: loss", epoch_loss, "val", vloss, vrec)


if __name__ == "__main__":
    os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
    sys.dont_write_bytecode = True
    lgconv_cases()
    harness()
