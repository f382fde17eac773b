"""Data-parallel Cluster-GCN training over one process per GPU (torch.distributed; backend
"nccl" is RCCL over xGMI on MI355X, "gloo" on CPU for tests).

The reference trains one Cluster-GCN part per step on one GPU (reference utils/train_test.py:
66-103 over data/dataset_handler.py:285's loader). Here each of W ranks takes a disjoint batch of
parts per step from an epoch permutation every rank derives from the same seed, runs forward +
BPR + backward locally, then the two dense embedding gradients ([U,d] and [I,d]) are summed
with one all_reduce each and divided by W, and every rank applies the identical
clip_grad_norm_(1) + Adam step, so the replicated tables stay bitwise identical.
With W = 1 this is exactly the reference step.

With the row-lazy optimizer (lgcn_amd.optim.RowLazyAdam) the dense all_reduce is replaced by
RowExchange: only the rows a step can make nonzero travel (one all_gather per step of packed
row records: ids and rows), every rank sums them in rank order, and every rank updates exactly
the union of the ranks' rows.
"""
from __future__ import annotations


import torch
import torch.distributed as dist


def device_collectives(group=None) -> bool:
    """True where the multi-GPU paths run their collectives on device tensors in stream order
    (backend "nccl" = RCCL): side streams, events, in-place views, no host staging. gloo runs the
    same calls on CUDA tensors too (tools/rccl_probe.py --backend gloo), so
    lgcn_amd.tuning's device_collectives=True sends a gloo run down that branch — how the
    ranks-on-one-GPU tests exercise the code the RCCL runs take, since RCCL refuses two ranks on
    one GPU."""
    from . import tuning

    if tuning.get().device_collectives:
        return True
    return dist.get_backend(group) == "nccl"


def dp_lr(lr: float, world: int) -> float:
    """The Adam learning rate for data-parallel training over `world` ranks: lr * sqrt(world).

    A data-parallel step averages `world` parts' gradients, so an epoch takes `world` times fewer
    (and less noisy) Adam steps than the reference's one-part-per-step loop (reference
    utils/train_test.py:86-101); at the reference's lr the model then trails it. Measured on the C1
    graph against the reference harness (tools/dp_lr_probe.py, profiles/r05zg_dp_lr/: |dRecall@20|
    / |dRecall@100| at W = 8, 5 epochs): lr x1 0.0015 / 0.0030 (Recall@100 outside the +-0.002
    band), x sqrt(8) 0.00015 / 0.00025, x8 0.0008 / 0.0008; sqrt(W) is also the closest at W = 2
    and 4 and at 10 epochs (all within 0.0005 on both metrics)."""
    return float(lr) * float(world) ** 0.5


def world_info():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def epoch_order(num_batches: int, seed: int, epoch: int) -> torch.Tensor:
    """The shared shuffled order of batches for one epoch (same on every rank)."""
    g = torch.Generator().manual_seed(seed * 1_000_003 + epoch)
    return torch.randperm(num_batches, generator=g)


def rank_share(num_batches: int, world: int, rank: int, seed: int, epoch: int) -> list[int]:
    """Rank r's batches for the epoch: order[r], order[r + W], ... — every rank gets the same number
    of steps (the last num_batches % W batches of the order are left for the next epoch's shuffle)."""
    order = epoch_order(num_batches, seed, epoch).tolist()
    steps = num_batches // world
    if steps == 0:
        raise ValueError(f"{num_batches} batches cannot feed {world} ranks")
    return [order[s * world + rank] for s in range(steps)]


def allreduce_grads(params, world: int) -> None:
    if world == 1:
        return
    for p in params:
        if p.grad is None:
            p.grad = torch.zeros_like(p)
        dist.all_reduce(p.grad, op=dist.ReduceOp.SUM)
        p.grad.div_(world)


def exchange_capacity(batches, num_users: int) -> int:
    """Slots per rank for the row-sparse gradient exchange: the most rows any batch's step can
    list (its touched rows plus one negative per (user, positive) triplet), agreed across ranks
    (all_gather needs equal sizes)."""
    cap = 0
    for b in batches:
        ei = b.edge_index
        n_t = int(torch.unique(ei).numel())
        B = int((ei[0] < num_users).sum())
        cap = max(cap, n_t + B)
    world, _ = world_info()
    if world > 1:
        t = torch.tensor([cap], dtype=torch.int64)
        if device_collectives():
            t = t.cuda()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        cap = int(t.item())
    return cap


class RowExchange:
    """Row-sparse DP gradient exchange for the row-lazy optimizer (csrc/lgcn_exchange.hip).

    Per step each rank packs its listed gradient rows into ONE record block (fp32 [cap*(d+2)]:
    the slot ids as int64 [cap] in the first 2*cap words, then the rows [cap, d]); the blocks are
    all-gathered in one collective (RCCL over xGMI; gloo in tests), the ids copied out contiguous,
    and every rank sums the rows per row in rank order and divides by W, so the union's gradient
    rows — and the clip norm and Adam update over them — are bitwise identical on every rank.
    Bytes per rank per step: cap * (4d + 8), against 4d * N for the dense all_reduce (C4: ~17k
    rows of 512 B vs 113 MB)."""

    def __init__(self, cap: int, N: int, d: int, device, world: int):
        # cap even: each rank's block (cap*(d+2) words) and its rows (after 2*cap words) stay
        # 16-byte aligned for the float4 kernels (d % 4 == 0)
        self.cap, self.N, self.d, self.world = int(cap) + int(cap) % 2, int(N), int(d), int(world)
        self.blk = self.cap * (self.d + 2)
        self.pack = torch.zeros(self.blk, dtype=torch.float32, device=device)
        self.ids = self.pack[:2 * self.cap].view(torch.int64)
        self.ids.fill_(-1)
        self.rows = self.pack[2 * self.cap:].view(self.cap, self.d)
        self.pack_all = torch.zeros(self.world * self.blk, dtype=torch.float32, device=device)
        self.ids_all = torch.full((self.world * self.cap,), -1, dtype=torch.int64, device=device)
        self.first = torch.zeros(self.world * self.cap, dtype=torch.uint8, device=device)
        self.claim = torch.full((self.N,), 2**31 - 1, dtype=torch.int32, device=device)
        self.bytes = 0  # received from peers over the run

    def rows_ptr(self) -> int:
        """device pointer of rank 0's rows in the gathered records."""
        return self.pack_all.data_ptr() + 8 * self.cap

    def unpack_ids(self) -> None:
        """ids_all[r*cap + j] = rank r's slot j id (captured with the step's second half)."""
        blocks = self.pack_all.view(self.world, self.blk)[:, :2 * self.cap].view(torch.int64)
        self.ids_all.view(self.world, self.cap).copy_(blocks)

    def gather(self) -> None:
        """The collective (eager, between the step's two captured halves): one per step."""
        self.bytes += (self.world - 1) * self.blk * 4
        if self.world == 1:
            self.pack_all.copy_(self.pack)
        elif device_collectives():
            dist.all_gather_into_tensor(self.pack_all, self.pack)
        else:
            dist.all_gather(list(self.pack_all.view(self.world, self.blk).unbind(0)), self.pack)


def user_exchange_capacity(batches, num_users: int) -> int:
    """Slots per rank for HybridExchange's user records: the most user rows any batch touches,
    agreed across ranks."""
    cap = 0
    for b in batches:
        cap = max(cap, int((torch.unique(b.edge_index) < num_users).sum()))
    world, _ = world_info()
    if world > 1:
        t = torch.tensor([cap], dtype=torch.int64)
        if device_collectives():
            t = t.cuda()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        cap = int(t.item())
    return cap


class HybridExchange(RowExchange):
    """Data-parallel exchange for LARGE batches (a structured graph's Cluster-GCN batches, where a
    step's B negatives cover nearly every item): the item gradient table is all_reduced densely —
    I x d floats, less than the sparse records of ~I distinct item rows plus their ids — and only
    the users' rows (each user is in one part, so one rank's batch, per epoch) travel as
    RowExchange record blocks. Every rank then steps the union of the users' rows and ALL item
    rows (an item without a gradient this step takes Adam's zero-gradient step, bitwise what the
    row-lazy replay would give it later). The item sums are the collective's (RCCL ring / gloo), not
    rank order: at W = 2 bitwise the replicated exchange (a + b == b + a), above it equal to
    rounding; every rank's tables stay bitwise identical (every rank receives the same sums).

    gi: the optimizer's item gradient table (RowLazyAdam.gi), zeroed by the step before it writes
    and summed in place."""

    dense_items = True

    def __init__(self, cap_users: int, num_users: int, gi: torch.Tensor, device, world: int):
        I, d = gi.shape
        super().__init__(cap_users, int(num_users) + int(I), d, device, world)
        self.U = int(num_users)
        self.gi = gi
        self.items_all = torch.arange(self.U, self.U + int(I), dtype=torch.int32, device=device)

    def gather(self) -> None:
        super().gather()  # the users' record blocks
        if self.world == 1:
            return
        self.bytes += int(2 * (self.world - 1) * self.gi.numel() * 4 // self.world)  # ring all_reduce
        dist.all_reduce(self.gi, op=dist.ReduceOp.SUM)


def train_epoch(model, optimizer, batches, device, seed: int = 0, epoch: int = 0, loss_fn=None,
                embed_fn=None, max_norm: float = 1.0) -> float:
    """One data-parallel epoch; returns the global edge-weighted mean loss (as reference train())."""
    from utils.train_test import bpr_loss, compute_embeddings

    loss_fn = loss_fn or bpr_loss
    embed_fn = embed_fn or compute_embeddings
    world, rank = world_info()
    model.train()
    params = list(model.parameters())
    acc = torch.zeros(2, dtype=torch.float64, device=device)  # [sum loss*w, sum w]
    for b in rank_share(len(batches), world, rank, seed, epoch):
        batch = batches[b].to(device)
        optimizer.zero_grad()
        loss = loss_fn(*embed_fn(model, batch, device))
        loss.backward()
        allreduce_grads(params, world)
        if getattr(optimizer, "fused_clip_norm", None) is None:
            torch.nn.utils.clip_grad_norm_(params, max_norm=max_norm)
        optimizer.step()
        w = batch.edge_index.shape[1]
        acc[0] += loss.detach().double() * w
        acc[1] += w
    if world > 1:
        dist.all_reduce(acc, op=dist.ReduceOp.SUM)
    tot = acc.cpu().tolist()
    return tot[0] / tot[1]
