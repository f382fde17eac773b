"""ORACLE — test infrastructure, not product code.

Only tests/ may import this module, and only as the checker. The product path (lgcn_amd,
models/, utils/) never calls it.

CPU restatement (numpy, float64 scores) of the reference's Recall@k
(reference utils/train_test.py:165-212, compute_recall_at_k, reached from evaluate :136-163):

  * candidates = cat(normalize(pos), normalize(neg)); normalize(x) = x / ||x||_2 per row (:53-64);
  * per sample (num_samples draws): picked = np.random.choice(num_users, sample_size,
    replace=False) (:187) — the same numpy global-RNG calls in the same order;
  * scores = normalize(users[picked]) @ candidates.T; top-k indices per row (torch.topk, :196);
    hits = number of those indices < P (the positive block, :192-199);
  * recall per user = hits / P in float32; per-sample mean in float32 (torch's CPU reduction,
    so the value is the reference's to the bit); summed in Python floats over samples and divided
    by num_samples (:201-209).

Scores here are float64, and ties at the k-th score take the lowest index first, so queries
whose k-th and (k+1)-th float64 scores are closer than fp32 rounding are "unseparated"
(`topk_hits(..., return_gap=True)` reports the gap): there, the reference's own torch.topk
order is rounding- and implementation-defined.
"""
from __future__ import annotations

import numpy as np


def normalize(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, dtype=np.float64)
    return x / np.sqrt((x * x).sum(axis=1, keepdims=True))


def topk_hits(queries: np.ndarray, pos: np.ndarray, neg: np.ndarray, k: int, return_gap: bool = False):
    """hits[q] = #positives among the k best candidates of query row q (reference :190-199)."""
    q = normalize(queries)
    c = np.concatenate([normalize(pos), normalize(neg)])
    P = pos.shape[0]
    if k > c.shape[0]:
        raise RuntimeError("selected index k out of range")
    s = q @ c.T
    # descending score, ascending index among equal scores
    order = np.lexsort((np.broadcast_to(np.arange(c.shape[0]), s.shape), -s), axis=1)
    top = order[:, :k]
    hits = (top < P).sum(axis=1)
    if not return_gap:
        return hits
    srt = np.take_along_axis(s, order, axis=1)
    gap = srt[:, k - 1] - (srt[:, k] if k < c.shape[0] else -np.inf)
    return hits, gap


def _mean_f32(v: np.ndarray) -> float:
    """torch's float32 mean of a CPU tensor (its reduction order), as the reference's .mean()."""
    import torch

    return torch.from_numpy(np.ascontiguousarray(v, dtype=np.float32)).mean().item()


def recall_at_k(embs, k: int = 20, num_samples: int = 10, sample_size: int = 100, return_detail: bool = False):
    """Reference compute_recall_at_k on numpy arrays; draws from np.random exactly as it does."""
    users, pos, neg = (np.asarray(e) for e in embs)
    P = pos.shape[0]
    total = 0.0
    detail = []
    for _ in range(num_samples):
        picked = np.random.choice(users.shape[0], sample_size, replace=False)
        hits, gap = topk_hits(users[picked], pos, neg, k, return_gap=True)
        per_user = hits.astype(np.float32) / np.float32(P)
        total += _mean_f32(per_user)
        detail.append((picked, hits, gap))
    r = total / num_samples
    return (r, detail) if return_detail else r
