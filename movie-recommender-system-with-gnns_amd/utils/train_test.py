"""Training / evaluation harness with the reference's API (reference utils/train_test.py:18-256).

Same functions, arguments and results as the reference:
  bpr_loss (:18-51) — cosine BPR ×10 softplus with L2 on layer-0 rows (coeff 5e-3);
  normalize_embedding (:53-64); train (:66-103) — one epoch over the cluster loader with
  Adam + clip_grad_norm_(1); compute_embeddings (:105-134); evaluate (:136-163) — loss and
  Recall@top_k on layer-0 rows; compute_recall_at_k (:165-212);
  train_model (:214-256) — epochs, best-recall checkpoint to best_model.pth.
Differences are in where the work runs, not in the numbers:
  * the per-step ``loss.item()`` host sync (:101) is replaced by a float64 accumulation on the
    device (the same double-precision sums), read once per epoch;
  * Recall@k keeps the reference's numpy sampling (np.random.choice, :187) but labels the top-k
    hits by index (< number of positives) instead of gathering from a [100, 2B] mask — the same
    0/1 values — and reads the per-sample means back once. On device tensors it runs the HIP
    kernels of lgcn_amd.recall (all samples in one pass, no [100, 2B] score matrix).
"""
from typing import Tuple

import numpy as np
import torch
from torch import optim

try:  # the reference shows a tqdm bar over epochs (:239); optional here
    from tqdm import tqdm
except ImportError:  # pragma: no cover
    def tqdm(x):
        return x

from utils.helpers import get_triplets_indices

torch.manual_seed(0)  # import-time seeding, as reference utils/train_test.py:12-16
torch.cuda.manual_seed(0)
torch.cuda.manual_seed_all(0)
torch.backends.cudnn.deterministic = True
torch.backends.cudnn.benchmark = False


def normalize_embedding(emb: torch.Tensor) -> torch.Tensor:
    """Row-wise L2 normalisation (reference :53-64)."""
    return emb / torch.norm(emb, p=2, dim=1, keepdim=True)


def bpr_loss(emb_users_final: torch.Tensor, emb_users: torch.Tensor,
             emb_pos_items_final: torch.Tensor, emb_pos_items: torch.Tensor,
             emb_neg_items_final: torch.Tensor, emb_neg_items: torch.Tensor,
             bpr_coeff: float = 5e-3) -> torch.Tensor:
    """-mean(softplus(10 (cos(u,p) - cos(u,n)))) / 10 + coeff * mean(|e_u|² + |e_p|² + |e_n|²)
    over the batch, cosines on the propagated rows, L2 on layer-0 rows (reference :18-51)."""
    squares = emb_users * emb_users + emb_pos_items * emb_pos_items + emb_neg_items * emb_neg_items
    reg_loss = bpr_coeff * squares.mean()
    u = normalize_embedding(emb_users_final)
    p = normalize_embedding(emb_pos_items_final)
    n = normalize_embedding(emb_neg_items_final)
    margin = torch.sum(u * p, dim=1) - torch.sum(u * n, dim=1)
    ranking = torch.mean(torch.nn.functional.softplus(10 * margin)) / 10.
    return -ranking + reg_loss


def compute_embeddings(model: torch.nn.Module, data, device) -> Tuple[torch.Tensor, ...]:
    """The six [B, d] row sets the loss needs: propagated and layer-0 rows of the batch's users,
    positives and sampled negatives (reference :105-134)."""
    users_final, items_final = model(data.edge_index)
    users_0, items_0 = model.user_embedding.weight, model.item_embedding.weight
    u, p, n = get_triplets_indices(data.edge_index, model.num_users, model.num_items, device)
    return (users_final[u], users_0[u],
            items_final[p], items_0[p],
            items_final[n], items_0[n])


# which step the last train() call ran: "fused" (lgcn_amd.harness) or "reference: <why not fused>"
LAST_TRAIN_PATH = None


def _reference_step(model, optimizer, batch, device):
    """One step of the reference loop (:86-101): (loss * edges as a device tensor, edges)."""
    batch = batch.to(device)
    optimizer.zero_grad()
    loss = bpr_loss(*compute_embeddings(model, batch, device))
    loss.backward()
    if getattr(optimizer, "fused_clip_norm", None) is None:
        torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1)
    optimizer.step()  # lgcn_amd.optim.FusedAdam(max_grad_norm=1) clips inside its step
    w = batch.edge_index.shape[1]
    return loss.detach().double() * w, w


def train(model: torch.nn.Module, optimizer: torch.optim.Optimizer, train_loader, device) -> float:
    """One epoch over the loader; returns the edge-weighted mean batch loss (reference :66-103).
    A HIP LightGCN with the reference's torch Adam runs the fused batch step (lgcn_amd.harness:
    HIP forward / BPR / backward and the exact row-lazy Adam, one hipGraph per batch) with the
    same negatives, loss and optimizer state; anything else runs the reference-style loop below —
    from the first batch the fused step cannot take to the epoch's end (the loader is iterated
    once, so a one-shot iterator loses no batch)."""
    global LAST_TRAIN_PATH
    model.train()
    why = "model not on a ROCm device"
    total_loss, total_w = None, 0
    batches = train_loader
    rest = None  # the batches the fused step read but did not take (the reference loop takes them)
    weight = getattr(getattr(model, "user_embedding", None), "weight", None)
    if weight is not None and weight.is_cuda:
        from lgcn_amd import harness

        why = harness.eligibility(model, optimizer)
        if why is None:
            batches = iter(train_loader)
            if hasattr(train_loader, "__len__"):
                batches = _Sized(batches, len(train_loader))
            total_loss, total_w, rest, steps = harness.train_epoch(model, optimizer, batches, device)
            if rest is None:
                LAST_TRAIN_PATH = "fused"
                if total_loss is None:
                    raise ZeroDivisionError("empty train loader")
                return total_loss.item() / total_w
            why = "a batch is not a bipartite user-item edge list"
            if steps:
                why = f"fused for {steps} batch(es), then reference from a batch that is not a bipartite user-item edge list"
    LAST_TRAIN_PATH = f"reference: {why}"
    for batch in (_chain(rest, batches) if rest is not None else batches):  # rest: read, not taken
        contrib, w = _reference_step(model, optimizer, batch, device)
        total_w += w
        total_loss = contrib if total_loss is None else total_loss + contrib
    if total_loss is None:
        raise ZeroDivisionError("empty train loader")
    return total_loss.item() / total_w


class _Sized:
    """An iterator that still reports the loader's len() (the harness sizes its caches by it)."""

    def __init__(self, it, n):
        self.it, self.n = it, n

    def __iter__(self):
        return self.it

    def __len__(self):
        return self.n


def _chain(first, rest):
    yield from first
    yield from rest


def compute_recall_at_k(embs, k: int = 20, num_samples: int = 10, sample_size: int = 100, picks=None) -> float:
    """Reference Recall@k (:165-212): sample_size random positive-edge rows as 'users', score
    them against every positive and negative row of the batch, count top-k hits among the
    positives, divide by the number of positives; mean over num_samples draws. picks (device
    path): the draws already started by lgcn_amd.recall.start_picks."""
    user_embs, pos_item_embs, neg_item_embs = embs
    if user_embs.is_cuda:  # HIP path: f32 MFMA scores + per-user top-k selection, no score matrix
        from lgcn_amd.recall import compute_recall_at_k as recall_hip

        return recall_hip(embs, k=k, num_samples=num_samples, sample_size=sample_size, picks=picks)
    num_pos = pos_item_embs.size(0)
    candidates = torch.cat((normalize_embedding(pos_item_embs), normalize_embedding(neg_item_embs))).t()
    per_sample = []
    for _ in range(num_samples):
        picked = np.random.choice(user_embs.size(0), sample_size, replace=False)
        scores = torch.mm(normalize_embedding(user_embs[picked]), candidates)
        _, top = torch.topk(scores, k, dim=1)
        hits = (top < num_pos).to(scores.dtype).sum(dim=1)
        per_sample.append((hits / num_pos).mean())
    means = torch.stack(per_sample).double().cpu().tolist()
    total = 0.0
    for m in means:
        total += m
    return total / num_samples


def evaluate(model: torch.nn.Module, test_data, device, top_k: int = 100):
    """(BPR loss, Recall@top_k on layer-0 rows) of one edge set (reference :136-163)."""
    model.eval()
    with torch.no_grad():
        test_data = test_data.to(device)
        embs = compute_embeddings(model, test_data, device)
        picks = None
        if embs[1].is_cuda:
            # numpy's user draws for Recall@k (host) overlap the loss (GPU); neither touches the
            # other's generator, so the draws and the loss are the sequential ones
            from lgcn_amd.recall import start_picks

            picks = start_picks(embs[1].size(0))
        try:
            test_loss = bpr_loss(*embs).item()
            recall_at_k = compute_recall_at_k((embs[1], embs[3], embs[5]), k=top_k, picks=picks)
        finally:
            if picks is not None:  # never leave the draws moving numpy's state after we return
                picks.thread.join()
    return test_loss, recall_at_k


def train_model(model: torch.nn.Module, train_loader, val_data, test_data, device, epochs: int = 1,
                lr: float = 0.001, checkpoint: str = "best_model.pth", fused_optimizer: bool = False):
    """Epoch loop with validation and best-recall checkpointing (reference :214-256).
    fused_optimizer=True swaps torch Adam + clip_grad_norm_ for the two-launch HIP FusedAdam."""
    hist_train_loss, hist_val_loss, hist_val_recall = [], [], []
    if fused_optimizer:
        from lgcn_amd.optim import FusedAdam

        optimizer = FusedAdam(model.parameters(), lr=lr, max_grad_norm=1)
    else:
        optimizer = optim.Adam(model.parameters(), lr=lr)
    best_recall = 0
    for epoch in tqdm(range(epochs)):
        loss = train(model, optimizer, train_loader, device)
        val_loss, recall_at_k = evaluate(model, val_data, device)
        hist_train_loss.append(loss)
        hist_val_loss.append(val_loss)
        hist_val_recall.append(recall_at_k)
        print(f"Epoch: {epoch:03d}, Train Loss: {loss:.4f}, Val Loss: {val_loss:.4f}, "
              f"Recall@k: {recall_at_k:.6f}, k=100")
        if recall_at_k > best_recall:
            best_recall = recall_at_k
            if checkpoint:
                torch.save(model.state_dict(), checkpoint)
    test_loss, recall_at_k = evaluate(model, test_data, device)
    print(f"Test Loss: {test_loss:.4f}, Recall@k: {recall_at_k:.6f}, k=100")
    return model, hist_train_loss, hist_val_loss, hist_val_recall
