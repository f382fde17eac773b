"""Recall parity when training runs on several GPUs (VERDICT r02 missing #3; BASELINE.json north
star: Recall@20 within +-0.002 of the reference), at BASELINE configs[0]'s size
(tests/dp_recall_worker.py: C1 graph, 16 Cluster-GCN parts, K = 2, d = 64, Adam 1e-3, clip 1,
5 epochs), 8 gloo ranks on the one GPU.

* Data parallel (lgcn_amd.distributed, row-sparse exchange): W disjoint parts per optimizer step,
  their gradients summed in rank order / W — so after the same epochs the model has taken W-times
  fewer, larger steps than the reference's one-part-per-step loop (reference
  utils/train_test.py:86-101 over data/dataset_handler.py:285). At the reference's lr that leaves
  Recall@20 0.0015 and Recall@100 0.0030 below it (outside the band); with the Adam lr scaled by
  sqrt(W) (lgcn_amd.distributed.dp_lr, bench.py's default for DP) both are within 0.0005
  (tools/dp_lr_probe.py), and both are held to +-0.002 here. bench.py's default --dp-mode ("auto")
  keeps "columns" at 2 ranks and takes the owner-sharded form of this mode from 4 ranks, where it
  is the only one projected to scale (tools/project_c4.py).
* Column-sharded (lgcn_amd.train_step.ColumnGroup, SURVEY §8e's parity-preserving alternative):
  every rank steps the reference's schedule on d / W columns; one all_reduce of the triplets'
  [B, 6] dot products and norms and one all_gather of the clip norm's partials per step. Its
  losses track the one-GPU run's to 1e-5 at every step, its tables after the first step agree per
  row to 1e-5, W = 1 is bitwise the unsharded step, and its Recall is held to +-0.002 of the
  reference harness (CPU oracle) and of the one-GPU run.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu

EPOCHS, PARTS = 5, 16


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_ranks(world, out, mode="dp", lr_scale=1.0, epochs=EPOCHS):
    port = str(_free_port())
    worker = str(ROOT / "tests" / "dp_recall_worker.py")
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", OMP_NUM_THREADS="1")
    procs = [subprocess.Popen([sys.executable, "-u", worker, str(r), str(world), port, out, str(epochs), str(PARTS),
                               mode, str(lr_scale)],
                              env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(world)]
    logs = []
    try:
        for p in procs:
            logs.append(p.communicate(timeout=300)[0])
    except subprocess.TimeoutExpired:
        for q in procs:
            q.kill()
        raise
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-3000:]
    with open(out) as f:
        rec = json.load(f)
    if mode not in ("dp", "hybrid"):
        rec["tables"] = torch.load(out + ".pt", weights_only=True)
    return rec


class _Batch:
    def __init__(self, ei):
        self.edge_index = ei

    def to(self, device):
        return _Batch(self.edge_index.to(device))


def _reference_harness(epochs=EPOCHS):
    """The reference loop on the CPU oracle model: one part per step, torch Adam(1e-3) +
    clip_grad_norm_(1), 5 epochs in the shuffled order, then Recall on the validation edges."""
    sys.path.insert(0, str(ROOT / "tests"))
    from dp_recall_worker import c1_split
    from oracle.lgconv_torch import OracleLightGCN
    from utils import train_test as TT

    U, I, lists, val = c1_split(PARTS)
    from lgcn_amd import distributed as D

    torch.manual_seed(0)
    ref = OracleLightGCN(U, I, num_layers=2, dim_h=64)
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    cpu = torch.device("cpu")
    torch.manual_seed(1)
    for epoch in range(epochs):
        order = D.rank_share(len(lists), 1, 0, seed=0, epoch=epoch)
        TT.train(ref, opt, [_Batch(torch.from_numpy(lists[b])) for b in order], cpu)
    with torch.no_grad():
        embs = TT.compute_embeddings(ref, _Batch(torch.from_numpy(val)), cpu)
        rec = {}
        for k in (20, 100):
            np.random.seed(5)
            rec[str(k)] = TT.compute_recall_at_k((embs[1], embs[3], embs[5]), k=k)
    return rec


def test_multi_gpu_training_recall(gpu, tmp_path):
    from parity import assert_rows_close

    ref = _reference_harness()
    from lgcn_amd.distributed import dp_lr

    dp8 = _run_ranks(8, str(tmp_path / "dp8.json"), "dp", lr_scale=dp_lr(1.0, 8))
    hy8 = _run_ranks(8, str(tmp_path / "hy8.json"), "hybrid", lr_scale=dp_lr(1.0, 8))
    plain = _run_ranks(1, str(tmp_path / "plain.json"), "plain")
    cols1 = _run_ranks(1, str(tmp_path / "cols1.json"), "cols")
    cols8 = _run_ranks(8, str(tmp_path / "cols8.json"), "cols")
    assert dp8["steps_per_rank"] == EPOCHS * (dp8["parts"] // 8)
    assert cols8["steps_per_rank"] == plain["steps_per_rank"] == EPOCHS * plain["parts"]
    # column split at W = 1 is the unsharded step, bitwise
    assert cols1["tables"]["losses"] == plain["tables"]["losses"]
    for a, b in zip(cols1["tables"]["final"], plain["tables"]["final"]):
        assert torch.equal(a, b)
    # W = 8 columns: every step's loss to 1e-5; the first step's gradient rows per row to 1e-5; the
    # tables after it per row to 1e-5 on every element whose gradient is clear of that bar (Adam's
    # first step is ~lr * sign(g): noise-level gradients may take either sign)
    worst = max(abs(a - b) / max(abs(b), 1e-12) for a, b in zip(cols8["tables"]["losses"], plain["tables"]["losses"]))
    assert worst <= 1e-5, worst
    ids8, g8 = cols8["tables"]["first_grads"]
    ids1, g1 = plain["tables"]["first_grads"]
    assert torch.equal(ids8, ids1)
    assert_rows_close(g8.numpy(), g1.numpy(), what="first-step gradient rows, column-sharded vs 1 GPU")
    full8 = torch.cat(cols8["tables"]["first"]).numpy()
    full1 = torch.cat(plain["tables"]["first"]).numpy()
    g1n = g1.numpy()
    settled = np.abs(g1n) > 1e-4 * np.abs(g1n).max(axis=1, keepdims=True)
    diff = np.where(settled, np.abs(full8[ids1.numpy()] - full1[ids1.numpy()]), 0.0)
    scale = np.abs(full1[ids1.numpy()]).max(axis=1)
    assert float((diff.max(axis=1) / scale).max()) <= 1e-5
    untouched = np.setdiff1d(np.arange(full1.shape[0]), ids1.numpy())
    assert np.array_equal(full8[untouched], full1[untouched])  # rows without a gradient do not move
    bad = []
    for k in ("20", "100"):
        line = [f"Recall@{k}: reference harness (CPU oracle, 1 part/step) {ref[k]:.5f}"]
        for name, r in (("fused 1 GPU", plain), ("column-sharded W=8", cols8), ("data-parallel W=8 lr x sqrt(8)", dp8),
                        ("hybrid DP W=8", hy8)):
            line.append(f"{name} {r['recall'][k]:.5f} (|d| {abs(r['recall'][k] - ref[k]):.5f})")
        print(" | ".join(line) + f"; bar 0.002; max per-step loss rel diff (cols W=8 vs 1 GPU) {worst:.2e}")
        for name, r in (("column-sharded W=8", cols8), ("fused 1 GPU", plain)):
            if abs(r["recall"][k] - ref[k]) > 0.002:
                bad.append((name, k, r["recall"][k], ref[k]))
        dp_d = abs(dp8["recall"][k] - ref[k])
        if dp_d > 0.002:
            bad.append(("data-parallel W=8, lr x sqrt(8)", k, dp8["recall"][k], ref[k]))
        if abs(hy8["recall"][k] - ref[k]) > 0.002:  # the same DP semantics, item sums in the collective's order
            bad.append(("hybrid DP W=8, lr x sqrt(8)", k, hy8["recall"][k], ref[k]))
        print(f"data-parallel W=8 (lr x sqrt(8)) Recall@{k}: |d| {dp_d:.5f} "
              f"{'inside' if dp_d <= 0.002 else 'OUTSIDE'} the +-0.002 band (asserted)")
        if abs(cols8["recall"][k] - plain["recall"][k]) > 0.002:
            bad.append(("cols W=8 vs 1 GPU", k))
    assert not bad, bad
