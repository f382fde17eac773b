"""Owner-sharded row optimizer for data-parallel Cluster-GCN training (C4): the row-lazy Adam's
state and updates split across the ranks instead of replicated.

The reference trains one part per step on one GPU (reference utils/train_test.py:86-101 over
data/dataset_handler.py:285). In data parallel (lgcn_amd.distributed), W ranks take disjoint
batches per step and must apply one Adam step to the rank-ordered mean of their gradients. The
replicated exchange (distributed.RowExchange) all-gathers every rank's gradient rows so every
rank can step the whole union: each rank RECEIVES W - 1 ranks' rows (C4: 7 x 9.3 MB per step).

Here row r is owned by rank r % W, which alone keeps its Adam state (exp_avg, exp_avg_sq, last
step) and applies its updates. Per step, on every rank:

  1. the batch's gradient rows go to their owners (one all_to_all: W destination blocks);
  2. each owner sums the rows it received in rank order and divides by W (the same kernels and
     association as RowExchange: lgcn_rows_mark_first + lgcn_rows_accumulate);
  3. clip_grad_norm_(max_norm): every owner sums the squares of its rows in the step's union, in
     row order over its owned rows (lgcn_row_grad_sqnorm: fixed block partials), the W partial
     arrays are all-gathered and every rank finishes the same sum in rank order, so the clip
     coefficient is identical on every rank (but summed in another order than RowExchange's);
  4. the owner applies the exact row-lazy Adam step to its rows of the union;
  5. rows for the NEXT step: its batch (a fixed function of the shared epoch order) and its
     negatives (drawn one step ahead) are known now, so the ids travel with step 1's blocks as
     requests; each owner catches the requested rows up to the new step and sends them back
     (a second all_to_all), and the requester writes them into its table.

So every row a step reads is current on the rank that reads it, the rows nobody reads stay stale
until sync() (every owner replays its rows, then one all_gather of the owned rows makes every
table current — what evaluation and checkpoints need), and without clipping the result is
bitwise that of RowExchange (same sums, same updates, same replays). Bytes received per rank per
step: the W - 1 peers' blocks of (gradient rows + request ids) plus their replies — each about
1/W of a rank's listed rows — instead of W - 1 ranks' whole lists.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from . import _ffi
from .distributed import device_collectives


def owner_capacity(batches, num_users: int, world: int, slack: float = 1.25, floor: int = 64,
                   num_items: int | None = None) -> int:
    """Slots per destination block (gradient rows, and request ids): the most touched rows any
    batch has on one owner plus its negatives' share — in expectation B / W with slack (uniform
    negatives over the items: Binomial(B, 1/W) never comes near 1.25x its mean + 64 at these
    sizes), and at most the owner's items (row r is owned by rank r % W: ceil(I / W) of them),
    since both lists carry each distinct row once (gradient rows: first occurrences; requests:
    lgcn_owner_pack_requests' claim) — pass num_items for that bound (a structured graph's large
    batches: planted C3 at W = 8, 29k -> 8.3k slots). Even, agreed across ranks. A full
    destination is flagged (check_overflow), never silently wrapped."""
    cap = 0
    for b in batches:
        ei = b.edge_index
        touched = torch.unique(ei)
        per_owner = torch.bincount(touched % world, minlength=world).max().item() if touched.numel() else 0
        B = int((ei[0] < num_users).sum())
        neg = int(np.ceil(B / world * slack)) + floor
        if num_items is not None:
            neg = min(neg, -(-int(num_items) // world))
        cap = max(cap, int(per_owner) + neg)
    if dist.is_available() and dist.is_initialized() and world > 1:
        t = torch.tensor([cap], dtype=torch.int64)
        if device_collectives():
            t = t.cuda()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        cap = int(t.item())
    return cap + cap % 2


class OwnerExchange:
    """Buffers and collectives of the owner-sharded exchange (csrc/lgcn_exchange.hip lgcn_owner_*).

    One send block per destination: [gradient ids (int64, 2*cap floats) | gradient rows cap x d |
    request ids (int64, 2*cap floats)], padded to a multiple of 4 floats."""

    def __init__(self, cap: int, N: int, d: int, device, world: int, rank: int, norm_parts: int):
        if cap % 2:
            raise ValueError("cap must be even (16-byte aligned rows)")
        self.cap = self.rcap = int(cap)
        self.N, self.d, self.world, self.rank = int(N), int(d), int(world), int(rank)
        self.req_off = 2 * self.cap + self.cap * self.d
        blk = self.req_off + 2 * self.rcap
        self.blk = blk + (-blk) % 4
        W = self.world
        self.send = torch.zeros(W * self.blk, dtype=torch.float32, device=device)
        self.recv = torch.zeros(W * self.blk, dtype=torch.float32, device=device)
        self.counts = torch.zeros(2 * W, dtype=torch.int32, device=device)
        self.overflow = torch.zeros(1, dtype=torch.int32, device=device)
        self.ids_all = torch.full((W * self.cap,), -1, dtype=torch.int64, device=device)
        self.first = torch.zeros(W * self.cap, dtype=torch.uint8, device=device)
        self.claim = torch.full((self.N,), 2**31 - 1, dtype=torch.int32, device=device)
        self.req_all = torch.full((W * self.rcap,), -1, dtype=torch.int64, device=device)
        self.req_valid = torch.zeros(W * self.rcap, dtype=torch.uint8, device=device)
        self.mine = torch.full((W * self.rcap,), -1, dtype=torch.int64, device=device)
        self.reply_send = torch.zeros(W * self.rcap * self.d, dtype=torch.float32, device=device)
        self.reply_recv = torch.zeros(W * self.rcap * self.d, dtype=torch.float32, device=device)
        # the rows this rank owns (row order: the clip norm's fixed sweep) and the union mask
        self.owned = torch.arange(self.rank, self.N, W, dtype=torch.int64, device=device)
        self.not_union = torch.ones(self.N, dtype=torch.uint8, device=device)
        self.norm_parts = int(norm_parts)
        if torch.device(device).type == "cuda":
            # lgcn_row_grad_sqnorm writes exactly this many block partials (no size argument)
            need = _ffi.load().lgcn_row_grad_norm_workspace_floats()
            if self.norm_parts != need:
                raise ValueError(f"OwnerExchange: norm_parts={self.norm_parts} != the kernel's {need} partials")
        self.partials = torch.zeros(self.norm_parts, dtype=torch.float32, device=device)
        self.partials_all = torch.zeros(W * self.norm_parts, dtype=torch.float32, device=device)
        # request dedupe (lgcn_owner_pack_requests' claim): -1, then one increasing stamp per call
        self.req_claim = torch.full((self.N,), -1, dtype=torch.int32, device=device)
        self.req_stamp = 0
        self.nccl = W > 1 and device_collectives()
        self.bytes = 0  # received from peers over the run (self blocks excluded)
        self.pending = None  # the batch state whose rows the last step requested

    # --- block views -------------------------------------------------------------------------
    def _blocks(self, buf: torch.Tensor) -> torch.Tensor:
        return buf.view(self.world, self.blk)

    def unpack(self) -> None:
        """ids_all / req_all from the received blocks (captured with the owner's half)."""
        b = self._blocks(self.recv)
        self.ids_all.view(self.world, self.cap).copy_(b[:, :2 * self.cap].view(torch.int64))
        self.req_all.view(self.world, self.rcap).copy_(
            b[:, self.req_off:self.req_off + 2 * self.rcap].view(torch.int64))
        torch.ge(self.req_all, 0, out=self.req_valid)

    def rows_ptr(self) -> int:
        """device pointer of rank 0's gradient rows in the received blocks."""
        return self.recv.data_ptr() + 8 * self.cap

    # --- collectives (eager, between captured pieces) ------------------------------------------
    def _all_to_all(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        if self.world == 1:
            out.copy_(inp)
        elif self.nccl:
            dist.all_to_all_single(out, inp)
        else:  # gloo: through host memory
            o = torch.empty(out.shape, dtype=out.dtype)
            dist.all_to_all_single(o, inp.cpu())
            out.copy_(o)

    def exchange_blocks(self) -> None:
        self._all_to_all(self.recv, self.send)
        self.bytes += (self.world - 1) * self.blk * 4

    def exchange_replies(self) -> None:
        self._all_to_all(self.reply_recv, self.reply_send)
        self.bytes += (self.world - 1) * self.rcap * self.d * 4

    def gather_partials(self) -> None:
        if self.world == 1:
            self.partials_all.copy_(self.partials)
        elif self.nccl:
            dist.all_gather_into_tensor(self.partials_all, self.partials)
        else:
            dist.all_gather(list(self.partials_all.view(self.world, -1).unbind(0)), self.partials)
        self.bytes += (self.world - 1) * self.norm_parts * 4

    def check_overflow(self) -> None:
        v = int(self.overflow.item())
        if v:
            raise RuntimeError(f"OwnerExchange: a destination block overflowed (flags {v}); raise the capacity")

    # --- sync ----------------------------------------------------------------------------------
    def all_gather_owned(self, uw: torch.Tensor, iw: torch.Tensor, U: int) -> None:
        """Every rank's owned rows into every table (after each owner replayed its rows)."""
        lib = _ffi.load()
        W, d = self.world, self.d
        per = (self.N + W - 1) // W
        ids = torch.full((W, per), -1, dtype=torch.int64, device=uw.device)
        for r in range(W):
            own = torch.arange(r, self.N, W, dtype=torch.int64, device=uw.device)
            ids[r, :own.numel()] = own
        mine = torch.zeros((per, d), dtype=torch.float32, device=uw.device)
        s = _ffi.stream_of(uw.device)
        _ffi.check(lib.lgcn_rows_gather(uw.data_ptr(), iw.data_ptr(), U, d, ids[self.rank].contiguous().data_ptr(),
                                        per, mine.data_ptr(), 0, s), "lgcn_rows_gather(owned)")
        every = torch.empty((W * per, d), dtype=torch.float32, device=uw.device)
        if W == 1:
            every.copy_(mine)
        elif self.nccl:
            dist.all_gather_into_tensor(every, mine)
        else:
            host = torch.empty((W * per, d), dtype=torch.float32)
            dist.all_gather(list(host.view(W, per, d).unbind(0)), mine.cpu())
            every.copy_(host)
        self.bytes += (W - 1) * per * d * 4
        _ffi.check(lib.lgcn_rows_gather(uw.data_ptr(), iw.data_ptr(), U, d, ids.view(-1).data_ptr(), W * per,
                                        every.data_ptr(), 1, s), "lgcn_rows_gather(scatter all)")
