"""The harness's train() on the fused batch step (reference utils/train_test.py:66-103).

The reference's train() runs, per Cluster-GCN batch: the LightGCN forward, the six row gathers and
the cosine BPR loss, autograd's backward, clip_grad_norm_(max_norm=1) and torch Adam's step over
both dense [U, d] / [I, d] tables. utils.train_test.train keeps that loop for anything it does not
recognise; when the call is one the fused step reproduces, it runs
lgcn_amd.train_step.FusedTrainStep (the HIP forward, lgcn_bpr_fused, the touched-rows backward) with
the exact row-lazy Adam (lgcn_amd.optim.RowLazyAdam) instead, each batch's step captured once in a
hipGraph and replayed — bench.py's C3 step, ~14x faster than the reference-style step.

Eligible (eligibility() returns None): a LightGCN of this package on a ROCm device, a plain
torch.optim.Adam over exactly its two tables (one param group, betas (0.9, 0.999), eps 1e-8, no
weight decay / amsgrad / maximize / capturable / differentiable), d in {16, ..., 512}, and batches
that are bipartite user-item edge lists (the reference's triplets pair the k-th user-source edge's
user with its item).
LGCN_HARNESS_FUSED=0 forces the reference-style step.

What the caller sees is what the reference loop leaves: the model's tables and the torch
optimizer's state (exp_avg, exp_avg_sq, step per table) after the epoch — the row-lazy Adam is
flushed and its moments written back at the end of every train() call and read in at the start of
the next, so the two paths can alternate. The numbers: the same negatives (the global generator's
torch.randint, drawn in the same order), the loss within 1e-5, the tables within 1e-5 per row
(the clip norm sums the same squares in another order; tests/test_gpu_harness.py). Not reproduced:
the parameters' .grad after the epoch (the fused step writes its gradient rows into the
optimizer's own tables, not .grad; the reference leaves the last batch's gradient there).
"""
from __future__ import annotations

import os
import weakref

import torch

from . import _ffi

_DIMS = (16, 32, 64, 128, 256, 512)


def enabled() -> bool:
    return os.environ.get("LGCN_HARNESS_FUSED", "1") != "0"


def eligibility(model, optimizer) -> str | None:
    """None when train(model, optimizer, ...) can run on the fused step, else the reason not."""
    if not enabled():
        return "LGCN_HARNESS_FUSED=0"
    for a in ("num_users", "num_items", "num_layers", "dim_h", "user_embedding", "item_embedding"):
        if not hasattr(model, a):
            return f"model has no {a} (not a LightGCN)"
    uw, iw = model.user_embedding.weight, model.item_embedding.weight
    if not (uw.is_cuda and iw.is_cuda):
        return "tables not on a ROCm device"
    if uw.dtype != torch.float32 or iw.dtype != torch.float32 or not (uw.is_contiguous() and iw.is_contiguous()):
        return "tables not contiguous fp32"
    if model.dim_h not in _DIMS:
        return f"d={model.dim_h} not in {_DIMS}"
    if type(optimizer) is not torch.optim.Adam:
        return f"optimizer {type(optimizer).__name__} is not torch.optim.Adam"
    if len(optimizer.param_groups) != 1:
        return "more than one param group"
    g = optimizer.param_groups[0]
    ps = g["params"]
    if len(ps) != 2 or {id(p) for p in ps} != {id(uw), id(iw)}:
        return "the param group is not exactly the two embedding tables"
    if tuple(g["betas"]) != (0.9, 0.999) or g["eps"] != 1e-8 or g["weight_decay"] != 0:
        return "betas / eps / weight_decay differ from the reference's Adam defaults"
    for flag in ("amsgrad", "maximize", "capturable", "differentiable"):
        if g.get(flag, False):
            return f"Adam({flag}=True)"
    if isinstance(g["lr"], torch.Tensor):
        return "tensor lr"
    return None


class _Fast:
    """The fused step and row-lazy Adam attached to one (model, torch optimizer) pair."""

    def __init__(self, model, optimizer):
        from .optim import RowLazyAdam
        from .train_step import FusedTrainStep

        g = optimizer.param_groups[0]
        self.model = model
        self.lr = float(g["lr"])
        uw, iw = model.user_embedding.weight, model.item_embedding.weight
        self.opt = RowLazyAdam(uw.data, iw.data, lr=self.lr, betas=(0.9, 0.999), eps=1e-8, max_grad_norm=1.0)
        from utils import helpers

        num_items, dev = model.num_items, uw.device
        # the negatives come from the harness's own sampler (reference utils/helpers.py:64-82):
        # the reference loop's draws, and whatever a caller substitutes for them
        self.step = FusedTrainStep(model, self.opt, lazy=True, graphs=True,
                                   neg_sampler=lambda pos: helpers.sample_negative(pos, num_items, dev))
        # device copies of the loader's batches (keyed by the host edge_index, held weakly), so a
        # batch keeps its plans and captured graph from epoch to epoch
        self.dev_batches: dict[int, tuple[weakref.ref, torch.Tensor]] = {}

    def device_edge_index(self, ei: torch.Tensor, device) -> torch.Tensor:
        if ei.is_cuda:
            return ei
        hit = self.dev_batches.get(id(ei))
        if hit is not None and hit[0]() is ei and hit[1].shape == ei.shape:
            return hit[1]
        d = ei.to(device)
        self.dev_batches[id(ei)] = (weakref.ref(ei), d)
        if len(self.dev_batches) > 4096:
            for k in [k for k, (r, _) in self.dev_batches.items() if r() is None]:
                self.dev_batches.pop(k)
        return d

    # --- torch optimizer state <-> row-lazy Adam -----------------------------------------------
    def load_state(self, optimizer) -> None:
        """Start from the torch optimizer's state (none yet: step 0, zero moments)."""
        g = optimizer.param_groups[0]
        if float(g["lr"]) != self.lr:  # an lr change between epochs: new step constants
            self.lr = float(g["lr"])
            self.opt.lr = self.lr
            lib = _ffi.load()
            _ffi.check(lib.lgcn_adam_consts(self.opt.consts.data_ptr(), 1, self.opt.max_steps + 1, self.lr, 0.9,
                                            0.999, _ffi.stream_of(self.opt.device)), "lgcn_adam_consts")
        uw, iw = self.model.user_embedding.weight, self.model.item_embedding.weight
        steps = None
        for i, p in enumerate((uw, iw)):
            st = optimizer.state.get(p, {})
            if "exp_avg" in st:
                self.opt.m[i].copy_(st["exp_avg"])
                self.opt.v[i].copy_(st["exp_avg_sq"])
                s = int(float(st["step"]))
            else:
                self.opt.m[i].zero_()
                self.opt.v[i].zero_()
                s = 0
            if steps is not None and s != steps:
                raise RuntimeError("the two tables' Adam step counts differ")
            steps = s
        self.opt.steps = steps
        self.opt.step_dev.fill_(steps)
        self.opt.last.fill_(steps)  # every row current at that step

    def store_state(self, optimizer) -> None:
        """Every row replayed up to date, the moments and step count written back."""
        self.step.sync()
        uw, iw = self.model.user_embedding.weight, self.model.item_embedding.weight
        for i, p in enumerate((uw, iw)):
            st = optimizer.state[p]
            if "exp_avg" in st and st["exp_avg"].shape == p.shape:
                st["exp_avg"].copy_(self.opt.m[i])
                st["exp_avg_sq"].copy_(self.opt.v[i])
            else:
                st["exp_avg"] = self.opt.m[i].clone(memory_format=torch.preserve_format)
                st["exp_avg_sq"] = self.opt.v[i].clone(memory_format=torch.preserve_format)
            st["step"] = torch.tensor(float(self.opt.steps), dtype=torch.float32)


_FAST: "weakref.WeakKeyDictionary[torch.optim.Optimizer, _Fast]" = weakref.WeakKeyDictionary()


def bipartite(ei: torch.Tensor, U: int) -> bool:
    """Every edge joins a user and an item, so the k-th user-source edge gives both the k-th user
    and the k-th positive (reference utils/helpers.py:84-102) — the fused step's triplets."""
    return bool(((ei[0] < U) == (ei[1] >= U)).all().item())


def train_epoch(model, optimizer, train_loader, device) -> tuple[float, int] | None:
    """One train() epoch on the fused step: (sum over batches of loss * edges, total edges), or None
    if a batch is not eligible before any step ran (the caller then runs the reference loop)."""
    fast = _FAST.get(optimizer)
    if fast is None or fast.model is not model:
        fast = _Fast(model, optimizer)
        _FAST[optimizer] = fast
    fast.load_state(optimizer)
    total, total_w = None, 0
    U = model.num_users
    bad = object()  # a batch the fused step cannot take

    def device_batches():
        for batch in train_loader:
            ei = fast.device_edge_index(batch.edge_index, device)
            st = fast.step._states.get(id(ei))
            yield bad if (st is None or st[0]() is not ei) and not bipartite(ei, U) else ei

    try:
        it = device_batches()
        ei = next(it, None)
        if ei is bad:
            return None  # nothing ran: the caller runs the reference loop
        while ei is not None:
            nxt = next(it, None)
            if nxt is bad:
                raise ValueError("train(): a batch is not a bipartite user-item edge list; run with "
                                 "LGCN_HARNESS_FUSED=0")
            loss = fast.step.step(_Batch(ei))
            w = int(ei.shape[1])
            total_w += w
            contrib = loss.detach().double() * w
            total = contrib if total is None else total + contrib
            ei = nxt
    finally:
        if total is not None:
            fast.store_state(optimizer)
    if total is None:
        raise ZeroDivisionError("empty train loader")
    return total.item(), total_w


class _Batch:
    def __init__(self, ei):
        self.edge_index = ei
