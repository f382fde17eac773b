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
lgcn_amd.tuning.set_tuning(harness_fused=False) forces the reference-style step.

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

import weakref

import torch


_DIMS = (16, 32, 64, 128, 256, 512)


def enabled() -> bool:
    from . import tuning

    return tuning.get().harness_fused


def eligibility(model, optimizer) -> str | None:
    """None when train(model, optimizer, ...) can run on the fused step, else the reason not."""
    if not enabled():
        return "tuning harness_fused=False"
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


# batch states kept per (model, optimizer) beyond one epoch's batches (lgcn_amd._cache LRU)
_MIN_STATES = 64
# first size of the row-lazy Adam's per-step constant table (16 B per step; grown by doubling)
_MIN_STEPS = 4096


class _Fast:
    """The fused step and row-lazy Adam attached to one (model, torch optimizer) pair."""

    def __init__(self, model, optimizer):
        from ._cache import ContentLRU
        from .optim import RowLazyAdam
        from .train_step import FusedTrainStep

        g = optimizer.param_groups[0]
        self.model = model
        self.lr = float(g["lr"])
        uw, iw = model.user_embedding.weight, model.item_embedding.weight
        self.opt = RowLazyAdam(uw.data, iw.data, lr=self.lr, betas=(0.9, 0.999), eps=1e-8, max_grad_norm=1.0,
                               max_steps=_MIN_STEPS)
        num_items, dev = model.num_items, uw.device
        # the epoch's sum of loss * edges (reference utils/train_test.py:101-103), added on the
        # device by each captured step (lgcn_loss_accumulate): no per-step torch ops
        self.loss_acc = torch.zeros(1, dtype=torch.float64, device=dev)
        # the negatives come from the harness's own sampler (reference utils/helpers.py:64-82):
        # the reference loop's draws, and whatever a caller substitutes for them
        self.step = FusedTrainStep(model, self.opt, lazy=True, graphs=True, max_entries=_MIN_STATES,
                                   neg_sampler=_Sampler(num_items, dev), loss_acc=self.loss_acc)
        # device copies of host batches by content, so a batch keeps its plans and captured graph
        # from epoch to epoch even when the loader collates a new tensor each time
        self.dev_batches = ContentLRU(_MIN_STATES)
        # batch contents already checked bipartite (an object / content hit skips the check)
        self.checked = ContentLRU(_MIN_STATES)

    def size_for(self, n_batches: int | None) -> None:
        """Caches for one epoch of n_batches (plus slack), constants for this epoch's steps; called
        at an epoch's start, when every row is current."""
        if n_batches:
            cap = max(_MIN_STATES, 2 * n_batches)
            for c in (self.step._states, self.dev_batches, self.checked):
                c.resize(max(cap, c.capacity))
            self.reserve(self.opt.steps + n_batches)

    def grow_caches(self, cap: int) -> None:
        for c in (self.step._states, self.dev_batches, self.checked):
            if c.capacity < cap:
                c.resize(cap)

    def reserve(self, steps: int) -> None:
        if self.opt.reserve(steps):
            self.step.drop_graphs()  # the captured steps read the old constant table

    def device_edge_index(self, ei: torch.Tensor, device) -> torch.Tensor:
        if ei.is_cuda:
            return ei
        return self.dev_batches.get(ei, lambda: ei.to(device))

    def eligible(self, ei: torch.Tensor, U: int) -> bool:
        """The batch is a bipartite user-item edge list (checked once per content)."""
        return bool(self.checked.get(ei, lambda: bipartite(ei, U)))

    # --- torch optimizer state <-> row-lazy Adam -----------------------------------------------
    def load_state(self, optimizer) -> None:
        """Start from the torch optimizer's state (none yet: step 0, zero moments)."""
        g = optimizer.param_groups[0]
        if float(g["lr"]) != self.lr:  # an lr change between epochs: new step constants
            # (every row is current here, so no past step is replayed with them)
            self.lr = float(g["lr"])
            self.opt.lr = self.lr
            self.opt.regenerate_consts()
        uw, iw = self.model.user_embedding.weight, self.model.item_embedding.weight
        steps = None
        for i, p in enumerate((uw, iw)):
            st = optimizer.state.get(p, {})
            if "exp_avg" in st:
                # the torch state holds these very tables after a store (aliased): nothing to copy
                if st["exp_avg"] is not self.opt.m[i]:
                    self.opt.m[i].copy_(st["exp_avg"])
                if st["exp_avg_sq"] is not self.opt.v[i]:
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
        """Every row replayed up to date, the moments and step count written back. The torch
        state's moments ARE the row-lazy optimizer's tables (set once, aliased): no per-epoch copy
        either way, and a torch Adam step on them (the reference loop between fused epochs)
        updates them in place. A state replaced from outside (load_state_dict) is copied from."""
        self.step.sync()
        uw, iw = self.model.user_embedding.weight, self.model.item_embedding.weight
        for i, p in enumerate((uw, iw)):
            st = optimizer.state[p]
            for key, t in (("exp_avg", self.opt.m[i]), ("exp_avg_sq", self.opt.v[i])):
                if st.get(key) is not t:
                    st[key] = t
            st["step"] = torch.tensor(float(self.opt.steps), dtype=torch.float32)


class _Sampler:
    """utils.helpers.sample_negative(pos, num_items, device) as the step's negatives sampler. While
    that function is the reference's own (not patched by a caller), draw_into writes the same
    torch.randint(0, I, (B,)) draw straight into the batch's buffer (out=: the same kernel on the same
    shape, so the same values and generator offsets) instead of drawing a new tensor and copying it."""

    def __init__(self, num_items: int, device):
        from utils import helpers

        self.helpers = helpers
        self.num_items, self.device = int(num_items), device

    def __call__(self, pos):
        return self.helpers.sample_negative(pos, self.num_items, self.device)

    def draw_into(self, out, pos) -> None:
        if self.helpers.sample_negative is self.helpers.REFERENCE_SAMPLE_NEGATIVE:
            torch.randint(0, self.num_items, (pos.shape[0],), device=self.device, out=out)
        else:
            out.copy_(self(pos))


_FAST: "weakref.WeakKeyDictionary[torch.optim.Optimizer, _Fast]" = weakref.WeakKeyDictionary()


def bipartite(ei: torch.Tensor, U: int) -> bool:
    """Every edge joins a user and an item, so the k-th user-source edge gives both the k-th user
    and the k-th positive (reference utils/helpers.py:84-102) — the fused step's triplets."""
    return bool(((ei[0] < U) == (ei[1] >= U)).all().item())


_END = object()


def train_epoch(model, optimizer, batches, device):
    """Run the fused step over the batches iterator until it ends or yields a batch the fused step
    cannot take (not a bipartite user-item edge list). Returns (sum over the fused batches of
    loss * edges as a device tensor or None, their total edges, the batches read but not taken —
    a list, or None —, fused steps run). The torch optimizer holds the row-lazy Adam's state
    whenever this returns, so the caller runs the reference loop over the returned batches and
    then the rest of the iterator (it is read once: one-shot loaders lose no batch).
    The loader is read one batch ahead: a device edge_index of the next batch has its content
    digest enqueued (lgcn_amd._cache.prefetch) before this step's work, so it is ready when that
    batch's state is looked up — a loader that collates new device tensors every epoch costs no
    host sync per step."""
    fast = _FAST.get(optimizer)
    if fast is None or fast.model is not model:
        fast = _Fast(model, optimizer)
        _FAST[optimizer] = fast
    try:
        n = len(batches)
    except TypeError:
        n = None
    fast.load_state(optimizer)
    fast.size_for(n)
    fast.loss_acc.zero_()
    total, total_w, steps, leftover = None, 0, 0, None
    U = model.num_users
    from ._cache import prefetch

    it = iter(batches)
    nxt = next(it, _END)
    try:
        while nxt is not _END:
            batch = nxt
            nxt = next(it, _END)
            if nxt is not _END and getattr(nxt.edge_index, "is_cuda", False):
                prefetch(nxt.edge_index)
            ei = fast.device_edge_index(batch.edge_index, device)
            if not fast.eligible(ei, U):
                leftover = [batch] + ([nxt] if nxt is not _END else [])
                break
            if n is None and 2 * (steps + 1) > fast.step._states.capacity:
                # a loader without len(): the batch caches grow with the batches seen (an epoch of
                # more distinct batches than they hold would miss on every step)
                fast.grow_caches(2 * fast.step._states.capacity)
            if fast.opt.steps + 1 > fast.opt.max_steps:  # a loader without len(): grow mid-epoch
                fast.step.sync()  # every row current before the constants are regenerated
                fast.reserve(fast.opt.steps + 1)
            fast.step.step(_Batch(ei))  # adds double(loss) * edges to fast.loss_acc on the device
            steps += 1
            total_w += int(ei.shape[1])
    finally:
        if steps:
            total = fast.loss_acc.clone()
            fast.store_state(optimizer)
    return total, total_w, leftover, steps


class _Batch:
    def __init__(self, ei):
        self.edge_index = ei
