"""Recall@k on the GPU: the reference's compute_recall_at_k (utils/train_test.py:165-212) as
three HIP launches per pass (csrc/lgcn_recall.hip), with no [Q, M] score matrix and one host
read per call.

    Qn = normalize(users[picked])               lgcn_normalize_rows (gathered, zero-padded)
    Cn = cat(normalize(pos), normalize(neg))    lgcn_normalize_rows x2
    thr = k-th best of a strided subset         lgcn_score_filter (dense) + lgcn_select_topk
    lists = scores >= thr                       lgcn_score_filter (f32 MFMA, all M)
    hits = positives in the top k               lgcn_select_topk

All num_samples x sample_size sampled users go through one pass (a query's hits do not depend on
the other queries), and the numpy draws are the reference's own calls in the same order.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _ffi

# candidates scored for the first thresholds (≈ k·M/subset survive the filter; lgcn_amd.tuning's
# recall_subset, default 16384) and the per-query list capacity (>= the subset: the first pass
# stores every subset score)
CAP_MIN = 16384


class _Workspace:
    def __init__(self):
        self.key = None

    def get(self, dev, Qpad, M, D, cap):
        key = (dev, Qpad, M, D, cap)
        if key != self.key:
            self.key = key
            self.Qn = torch.empty((Qpad, D), dtype=torch.float32, device=dev)
            self.Cn = torch.empty((max(M, 1), D), dtype=torch.float32, device=dev)
            self.lkey = torch.empty((Qpad, cap), dtype=torch.int32, device=dev)
            self.lidx = torch.empty((Qpad, cap), dtype=torch.int32, device=dev)
            self.lcnt = torch.zeros(Qpad, dtype=torch.int32, device=dev)
            self.thr = torch.empty(Qpad, dtype=torch.int32, device=dev)
            self.hits = torch.empty(Qpad, dtype=torch.int32, device=dev)
        return self


_WS = _Workspace()


def _normalize_into(lib, x: torch.Tensor, idx, rows: int, out_ptr: int, D: int, out_rows: int, stream):
    if x.dim() != 2 or x.dtype != torch.float32 or x.stride(1) != 1:
        raise TypeError("recall: embeddings must be 2-D fp32 with unit column stride")
    _ffi.check(lib.lgcn_normalize_rows(x.data_ptr() if x.numel() else None, idx, rows, x.stride(0), x.shape[1],
                                       out_ptr, D, out_rows, stream), "lgcn_normalize_rows")


def topk_hits(users: torch.Tensor, picked: torch.Tensor, pos: torch.Tensor, neg: torch.Tensor, k: int,
              cap: int | None = None, subset: int | None = None, ties: str | None = None) -> torch.Tensor:
    """hits[q] = number of positives (rows of ``pos``) among the top-k cosine scores of
    users[picked[q]] against cat(pos, neg); int32 [Q] on the device.
    ties (default lgcn_amd.tuning's recall_ties): which of several EQUAL scores at the k-th place
    count — "index": the lowest candidate indices, i.e. the positives (torch.topk on a GPU, the
    reference's device when it has one); "cpu": the slots CPU torch.topk fills (libstdc++
    partial_sort / nth_element, lgcn_select_topk_stl). They differ only where a candidate row
    repeats another (an item that is one edge's positive and another's sampled negative)."""
    from . import tuning

    ties = tuning.get().recall_ties if ties is None else ties
    if ties not in ("index", "cpu"):
        raise ValueError(f"recall: ties must be 'index' or 'cpu', got {ties!r}")
    subset = tuning.get().recall_subset if subset is None else int(subset)
    cap = max(subset, CAP_MIN) if cap is None else int(cap)
    lib = _ffi.load()
    dev = users.device
    for t in (users, pos, neg):
        _ffi.require_device(t, "recall")
    d = users.shape[1]
    if pos.shape[1] != d or neg.shape[1] != d:
        raise ValueError("recall: users, positives and negatives must have the same width")
    P, Nn = pos.shape[0], neg.shape[0]
    M = P + Nn
    if k > M:
        raise RuntimeError("selected index k out of range")
    if k > cap:
        raise ValueError(f"recall: k={k} exceeds the list capacity {cap}")
    Dv, qm = ctypes.c_int32(0), ctypes.c_int32(0)
    _ffi.check(lib.lgcn_recall_width(d, ctypes.byref(Dv), ctypes.byref(qm)), "lgcn_recall_width")
    D, qmul = Dv.value, qm.value
    picked = picked.to(device=dev, dtype=torch.int64).contiguous()
    Q = picked.numel()
    Qpad = max(qmul, (Q + qmul - 1) // qmul * qmul)
    ws = _WS.get(dev, Qpad, M, D, cap)
    s = _ffi.stream_of(dev)
    _normalize_into(lib, users, picked.data_ptr(), Q, ws.Qn.data_ptr(), D, Qpad, s)
    _normalize_into(lib, pos, None, P, ws.Cn.data_ptr(), D, P, s)
    _normalize_into(lib, neg, None, Nn, ws.Cn.data_ptr() + P * D * 4, D, Nn, s)
    if ties == "cpu":
        return _hits_cpu_ties(lib, ws, M, D, k, P, Q, Qpad, qmul, s)
    # first thresholds: the k-th best of a strided subset (a lower bound of the true k-th best)
    stride = max(1, -(-M // min(subset, cap)))
    S = -(-M // stride)
    _ffi.check(lib.lgcn_score_filter(ws.Qn.data_ptr(), Qpad, Q, ws.Cn.data_ptr(), S, stride, D, None,
                                     ws.lkey.data_ptr(), ws.lidx.data_ptr(), None, cap, s), "lgcn_score_filter")
    _ffi.check(lib.lgcn_select_topk(ws.lkey.data_ptr(), ws.lidx.data_ptr(), None, S, cap, k, P, Qpad, Q,
                                    ws.thr.data_ptr(), None, s), "lgcn_select_topk")
    for _ in range(8):
        ws.lcnt.zero_()
        _ffi.check(lib.lgcn_score_filter(ws.Qn.data_ptr(), Qpad, Q, ws.Cn.data_ptr(), M, 1, D, ws.thr.data_ptr(),
                                         ws.lkey.data_ptr(), ws.lidx.data_ptr(), ws.lcnt.data_ptr(), cap, s),
                   "lgcn_score_filter")
        if int(ws.lcnt[:Q].max().item()) <= cap:
            _ffi.check(lib.lgcn_select_topk(ws.lkey.data_ptr(), ws.lidx.data_ptr(), ws.lcnt.data_ptr(), 0, cap, k,
                                            P, Qpad, Q, None, ws.hits.data_ptr(), s), "lgcn_select_topk")
            return ws.hits[:Q].clone()
        # a list overflowed: its kept entries are real candidates, so their k-th best is a valid,
        # tighter threshold; filter again
        _ffi.check(lib.lgcn_select_topk(ws.lkey.data_ptr(), ws.lidx.data_ptr(), ws.lcnt.data_ptr(), 0, cap, k,
                                        P, Qpad, Q, ws.thr.data_ptr(), None, s), "lgcn_select_topk")
    raise RuntimeError("recall: candidate lists kept overflowing (scores too concentrated for the capacity)")


# dense score rows of one query block in the "cpu" tie mode (8 bytes per score: key + index)
STL_BLOCK_BYTES = 1 << 30


def _hits_cpu_ties(lib, ws, M: int, D: int, k: int, P: int, Q: int, Qpad: int, qmul: int, s) -> torch.Tensor:
    """topk_hits with CPU torch.topk's tie rule: each query block's scores are written densely in
    candidate order (lgcn_score_filter, dense mode — the same f32 MFMA scores as the filtered
    path), then lgcn_select_topk_stl replays libstdc++'s selection on every row."""
    blk = max(qmul, (STL_BLOCK_BYTES // (8 * max(M, 1))) // qmul * qmul)
    blk = min(blk, Qpad)
    dev = ws.Qn.device
    keys = torch.empty((blk, M), dtype=torch.int32, device=dev)
    idx = torch.empty((blk, M), dtype=torch.int32, device=dev)
    hits = torch.empty(Qpad, dtype=torch.int32, device=dev)
    for q0 in range(0, Qpad, blk):
        nb = min(blk, Qpad - q0)
        qv = max(0, min(nb, Q - q0))
        qptr = ws.Qn.data_ptr() + q0 * D * 4
        _ffi.check(lib.lgcn_score_filter(qptr, nb, qv, ws.Cn.data_ptr(), M, 1, D, None, keys.data_ptr(),
                                         idx.data_ptr(), None, M, s), "lgcn_score_filter(dense)")
        _ffi.check(lib.lgcn_select_topk_stl(keys.data_ptr(), idx.data_ptr(), M, M, k, P, nb, qv,
                                            hits.data_ptr() + q0 * 4, s), "lgcn_select_topk_stl")
    return hits[:Q].clone()


def legacy_choice(n: int, size: int, draws: int) -> np.ndarray:
    """``draws`` consecutive np.random.choice(n, size, replace=False) calls on numpy's global
    legacy generator (reference utils/train_test.py:187), as one [draws, size] int64 array: the
    same picks and the same generator state afterwards (lgcn_legacy_choice, host C++)."""
    state = np.random.get_state()
    if state[0] != "MT19937" or size > n or n <= 0 or size < 0 or n > 2**31 - 1:
        return np.stack([np.random.choice(n, size, replace=False) for _ in range(draws)])
    key = np.array(state[1], dtype=np.uint32)
    pos = ctypes.c_int32(int(state[2]))
    out = np.empty((draws, size), dtype=np.int64)
    rc = _ffi.load().lgcn_legacy_choice(key.ctypes.data, ctypes.byref(pos), n, size, draws, out.ctypes.data)
    if rc == _ffi.E_UNSUPPORTED:  # no worker thread / memory: numpy's own draws (the state is untouched)
        return np.stack([np.random.choice(n, size, replace=False) for _ in range(draws)])
    _ffi.check(rc, "lgcn_legacy_choice")
    np.random.set_state(("MT19937", key, pos.value, state[3], state[4]))
    return out


class _Picks:
    """legacy_choice on a host thread (the C++ call releases the GIL), so the draws overlap GPU
    work the caller issues meanwhile — which must not use numpy's global generator."""

    def __init__(self, n: int, size: int, draws: int):
        import threading

        self.args, self.out, self.err = (n, size, draws), None, None
        self.thread = threading.Thread(target=self._run, daemon=True)
        self.thread.start()

    def _run(self):
        try:
            self.out = legacy_choice(*self.args)
        except BaseException as e:  # noqa: BLE001 — re-raised in result()
            self.err = e

    def result(self) -> np.ndarray:
        self.thread.join()
        if self.err is not None:
            raise self.err
        return self.out


def start_picks(n: int, sample_size: int = 100, num_samples: int = 10) -> _Picks:
    """Start compute_recall_at_k's user draws (numpy's, in the reference's order) in the background."""
    return _Picks(n, sample_size, num_samples)


def compute_recall_at_k(embs, k: int = 20, num_samples: int = 10, sample_size: int = 100,
                        picks: _Picks | None = None) -> float:
    """The reference's compute_recall_at_k (utils/train_test.py:165-212) on device tensors.
    picks: the draws already started by start_picks(users, sample_size, num_samples)."""
    user_embs, pos_item_embs, neg_item_embs = embs
    num_pos = pos_item_embs.size(0)
    if picks is not None:
        if picks.args != (user_embs.size(0), sample_size, num_samples):
            raise ValueError(f"recall: picks were started for {picks.args}")
        picked = picks.result().reshape(-1)
    else:
        picked = legacy_choice(user_embs.size(0), sample_size, num_samples).reshape(-1)
    hits = topk_hits(user_embs, torch.from_numpy(picked), pos_item_embs, neg_item_embs, k)
    hits = hits.cpu()  # the one host read of the call
    if int(hits.min()) < 0:
        raise RuntimeError("recall: a query ranked fewer than k candidates")
    # the reference's float32 arithmetic on the host, per sample as it runs it (hits / P, then a
    # 1-D CPU mean): equal hit counts give the CPU reference's value to the bit
    per_user = hits.to(torch.float32) / num_pos
    total = 0.0
    for row in per_user.view(num_samples, sample_size):
        total += row.contiguous().mean().item()
    return total / num_samples
