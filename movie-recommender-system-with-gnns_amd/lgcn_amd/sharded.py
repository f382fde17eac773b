"""Sharded full-graph propagation over W GPUs (SURVEY.md §8e (i)+(ii); BASELINE.json's headline
"edges propagated/sec (K=3, d=64) at 1/2/4/8 GPUs" on configs[1]): an R x F grid of ranks,
R row groups (below) times F column groups (``ShardGrid``: each column group propagates its
d / F columns of every row it owns, with no exchange between column groups).

One graph, one K-layer LightGCN forward (reference models/light_gcn.py:28-40), split over W
ranks by DESTINATION rows; the total work is fixed (strong scaling):

* Ownership. Rank r owns one contiguous range of the user rows and one of the item rows, cut so
  every rank carries about the same number of in-edges (``balanced_bounds``). Every rank keeps
  the whole embedding table and the whole graph (it gathers from every source row).
* Padded layout. Rank r's rows sit at [r*cu, r*cu + n_r) of a padded user block of W*cu rows and
  at W*cu + [r*ci, r*ci + m_r) of a padded item block of W*ci rows (cu, ci = the largest range),
  so one layer's rows of every rank land with one ``all_gather_into_tensor`` per block (equal
  chunks, no copy). Node ids are remapped by ``RowShards.padmap``, which is strictly increasing:
  every row keeps its neighbours in the same order, so its sum is the same chain of additions as
  on one GPU. Schedules: with one row group (R = 1, columns split only) a rank runs the one-GPU
  schedule itself (the source-slice bounds of the full width, mapped the same way), so hub rows
  are cut into the same chunks and the result is BITWISE the one-GPU result. With R > 1 a rank
  runs the plain item schedule (one launch per half-layer, ``rank_chunk``): bitwise the one-GPU
  plain schedule at that chunk, and within 1e-5 of the default (sliced) one, whose hub rows are
  chunked at slice boundaries too.
* Exchange overlapped with compute (bipartite graphs: every edge joins a user and an item).
  User rows gather only item rows and item rows only user rows, so a layer splits into two
  halves that share no row: A = the user-source slices (writes the item rows), B = the
  item-source slices (writes the user rows). Layer k runs A,B (k odd) or B,A (k even): each half
  reads the block whose all_gather was started first, and the block a half writes is all-gathered
  (RCCL, on a side stream) while the next half computes. Only layers 1..K-1 are exchanged; the
  final embedding stays row-sharded (each rank holds its own rows of the output).
* Non-bipartite graphs run each layer as one piece and exchange both blocks after it.

Host-side logic (``RowShards``, ``propagate_forward_sharded``) is device-agnostic so the gloo
CPU tests can drive the layer/exchange schedule; the kernels are the same lgcn_spmm* launches as
the one-GPU path (lgcn_amd.propagate.spmm).
"""
from __future__ import annotations

import dataclasses

import numpy as np
import torch

from . import _ffi
from .distributed import device_collectives

ROW_COST = 4  # a row's epilogue (acc/e/y traffic) costs about as much as this many gathered edges


def balanced_bounds(weight: np.ndarray, W: int) -> np.ndarray:
    """W+1 cut points over len(weight) rows: contiguous ranges of about equal weight."""
    weight = np.asarray(weight, dtype=np.float64)
    cs = np.concatenate([[0.0], np.cumsum(weight)])
    cuts = np.searchsorted(cs, cs[-1] * np.arange(1, W) / W, side="left")
    out = np.concatenate([[0], cuts, [weight.size]]).astype(np.int64)
    return np.maximum.accumulate(out)


@dataclasses.dataclass
class RowShards:
    """Ownership of the N = U + I destination rows by W ranks, and the padded id layout."""

    W: int
    U: int
    I: int
    ub: np.ndarray  # int64[W+1] user-row bounds (ids 0..U)
    ib: np.ndarray  # int64[W+1] item-row bounds (item-local ids 0..I)

    @classmethod
    def build(cls, in_degree: np.ndarray, U: int, W: int) -> "RowShards":
        deg = np.asarray(in_degree, dtype=np.int64)
        I = deg.size - U
        if U < 0 or I < 0 or W < 1:
            raise ValueError(f"bad shard request U={U} N={deg.size} W={W}")
        return cls(W, U, I, balanced_bounds(deg[:U] + ROW_COST, W), balanced_bounds(deg[U:] + ROW_COST, W))

    @property
    def N(self) -> int:
        return self.U + self.I

    @property
    def cu(self) -> int:
        return int(np.diff(self.ub).max()) if self.W else 0

    @property
    def ci(self) -> int:
        return int(np.diff(self.ib).max()) if self.W else 0

    @property
    def side(self) -> int:
        """First padded id of the item block."""
        return self.W * self.cu

    @property
    def NP(self) -> int:
        return self.W * (self.cu + self.ci)

    def padmap(self) -> np.ndarray:
        """int64[N]: original node id -> padded id (strictly increasing)."""
        out = np.empty(self.N, dtype=np.int64)
        for r in range(self.W):
            a, b = self.ub[r], self.ub[r + 1]
            out[a:b] = r * self.cu + np.arange(b - a)
            a, b = self.ib[r], self.ib[r + 1]
            out[self.U + a:self.U + b] = self.side + r * self.ci + np.arange(b - a)
        return out

    def user_rows(self, r: int) -> tuple[int, int]:
        lo = r * self.cu
        return lo, lo + int(self.ub[r + 1] - self.ub[r])

    def item_rows(self, r: int) -> tuple[int, int]:
        lo = self.side + r * self.ci
        return lo, lo + int(self.ib[r + 1] - self.ib[r])

    def block(self, b: str) -> tuple[int, int]:
        """(first padded row, rows per rank) of block 'u' (users) or 'i' (items)."""
        return (0, self.cu) if b == "u" else (self.side, self.ci)

    def owned_mask(self, r: int, blocks: str = "ui") -> np.ndarray:
        m = np.zeros(self.NP, dtype=np.uint8)
        if "u" in blocks:
            a, b = self.user_rows(r)
            m[a:b] = 1
        if "i" in blocks:
            a, b = self.item_rows(r)
            m[a:b] = 1
        return m

    def pad_bounds(self, bounds) -> list[int]:
        """Source-slice bounds (original ids, 0..N) in padded ids: each source keeps its slice."""
        pm = self.padmap()
        return [int(pm[b]) if b < self.N else self.NP for b in bounds]

    def to_padded(self, user_w: torch.Tensor, item_w: torch.Tensor) -> torch.Tensor:
        """The [NP, d] padded table of (user_w, item_w); padding rows are zero."""
        d = user_w.shape[1]
        out = torch.zeros((self.NP, d), dtype=user_w.dtype, device=user_w.device)
        pm = torch.from_numpy(self.padmap()).to(user_w.device)
        out[pm[: self.U]] = user_w
        out[pm[self.U:]] = item_w
        return out

    def from_padded(self, xp: torch.Tensor) -> torch.Tensor:
        """[N, d] rows of a padded table, in original id order."""
        return xp[torch.from_numpy(self.padmap()).to(xp.device)]


def rank_chunk(chunk: int, R: int) -> int:
    """Hub chunk of a rank's schedule: the one-GPU chunk with one row group (same schedule as one
    GPU, so bitwise its result); with R > 1 the plain schedule at min(chunk, RANK_CHUNK) (a
    shorter longest chain per launch; per-rank K=3 step at 8x1: 0.253 ms at 256, 0.246 at 128)."""
    from .plan import RANK_CHUNK

    return int(chunk) if R == 1 else min(int(chunk), RANK_CHUNK)


MIN_COLS = 32  # a column share narrower than 128 B rows stops cutting gather requests per edge


def grid_shape(world: int, d: int) -> tuple[int, int]:
    """(R row groups, F column groups), R * F = world: the fixed shape ShardGrid.build uses when
    none is given (bench.py instead times every grid_candidates grid and runs the fastest). Two
    column groups whenever the world is even and d / 2 >= MIN_COLS, the rest rows: columns need
    no exchange, and a 128-B row is one gather request instead of two (C2, one GPU, K=3:
    1.27 ms at d = 64, 0.74 at d = 32, 0.61 at d = 16, 0.77 at d = 8, profiles/r02x_cm/)."""
    if world >= 2 and world % 2 == 0 and d % 2 == 0 and d // 2 >= MIN_COLS and (d // 2) % 4 == 0:
        return world // 2, 2
    return world, 1


def grid_candidates(world: int, d: int, bipartite: bool = True,
                    p2p: bool = True) -> list[tuple[int, int, str | None]]:
    """(R, F, exchange mode) grids bench.py times before it picks one for a world of ranks (mode
    "reduce" — users sharded, item rows all-reduced — for every R > 1 of a bipartite graph): every
    column split F | world with d / F a multiple of 4 and >= 8; the rows-only grid (F = 1) when no
    column split exists or when world >= 4 — it moves the most bytes in total, but over R - 1 links
    at once, so its bytes per xGMI link match the column-split grids' (C2 at N = 8: ~14 MB per link
    per step for 8 x 1, 4 x 2 and 2 x 4) at the least compute per rank; both exchange modes where a
    row group has three or more ranks (an all_gather and direct peer sends differ there), none with
    R = 1. p2p=False: without the peer-send candidates."""
    out = []
    for F in range(world, 0, -1):
        if world % F or d % F or (d // F) % 4 or d // F < 8:
            continue
        R = world // F
        if R == 1:
            out.append((R, F, None))
        else:
            out += [(R, F, m) for m in (EXCHANGE_MODES if R >= 3 else EXCHANGE_MODES[:1])]
            if bipartite:  # users sharded, item rows all-reduced (ReducePlan), overlapped or fused order,
                # by RCCL's all_reduce or by all_to_all + ordered sums + all_gather (ItemReducer "a2a")
                out += [(R, F, "reduce"), (R, F, "reduce-fused"), (R, F, "reduce-a2a"), (R, F, "reduce-a2a-fused")]
    if any(F > 1 for _, F, _ in out) and world < 4:
        out = [c for c in out if c[1] > 1]
    # the peer-send candidates last: batch_isend_irecv is the one exchange outside RCCL's plain
    # collectives, so the log holds every plain candidate's time before them (a candidate that
    # raises is skipped either way; one that hangs ends the run at the process-group timeout)
    return [c for c in out if c[2] != "p2p"] + ([c for c in out if c[2] == "p2p"] if p2p else [])


@dataclasses.dataclass
class ShardGrid:
    """Rank r of an R x F grid: row group r // F (RowShards rank), column group r % F (columns
    [c0, c1) of the tables). Ranks of one column group exchange their rows (an all_gather over R
    ranks); column groups never exchange anything."""

    world: int
    rank: int
    R: int
    F: int
    d: int

    @classmethod
    def build(cls, world: int, rank: int, d: int, R: int | None = None, F: int | None = None) -> "ShardGrid":
        if R is None or F is None:
            R, F = grid_shape(world, d)
        if R * F != world or d % F or (d // F) % 4:
            raise ValueError(f"bad shard grid {R}x{F} for world {world}, d {d}")
        return cls(world, rank, R, F, d)

    @property
    def row_group(self) -> int:
        return self.rank // self.F

    @property
    def col_group(self) -> int:
        return self.rank % self.F

    @property
    def cols(self) -> tuple[int, int]:
        w = self.d // self.F
        return self.col_group * w, (self.col_group + 1) * w

    @property
    def members(self) -> list[int]:
        """Global ranks of this rank's column group, in row-group order (the exchange peers)."""
        return [self.col_group + self.F * i for i in range(self.R)]

    def exchange_group(self, dist):
        """The process group of this rank's column group (None = the default group when F = 1).
        Every rank must call this (new_group is collective over the world)."""
        if self.F == 1:
            return None
        mine = None
        for c in range(self.F):
            g = dist.new_group(ranks=[c + self.F * i for i in range(self.R)])
            if c == self.col_group:
                mine = g
        return mine


@dataclasses.dataclass
class Half:
    """One piece of a layer: the schedule of the rows it writes and the blocks it reads/writes."""

    direction: object  # CsrDirection | SlicedDirection (device) or a test stand-in
    reads: str         # 'u', 'i' or 'ui'
    writes: str
    partial: torch.Tensor | None = None


class ShardedPlan:
    """Rank `rank`'s propagation plan of a row-sharded graph: the whole (padded) CSR with gcn_norm
    weights from the whole graph's degrees, and the schedules of its own rows, per half."""

    def __init__(self, edge_index: torch.Tensor, shards: RowShards, rank: int, d: int, chunk: int | None = None,
                 slice_d: int | None = None):
        """d: the width this rank propagates (its column share); slice_d: the width whose one-GPU
        slicing decision and bounds are used (default d: the one-GPU plan at the share's width,
        whose result the share then is bitwise; the full width keeps the full-width segments and
        hub chunks instead, at 5-15 % more time for narrow shares, profiles/r02x_cm/)."""
        from .plan import DEFAULT_CHUNK, CsrDirection, _build_direction, _schedule, slice_bytes_for, sliced_chunk
        from .sliced import build_sliced, slice_bounds

        _ffi.require_device(edge_index, "ShardedPlan")
        if edge_index.dim() != 2 or edge_index.shape[0] != 2 or edge_index.dtype != torch.int64:
            raise ValueError("edge_index must be int64 [2, E]")
        self.shards, self.rank, self.d = shards, int(rank), int(d)
        self.chunk = rank_chunk(int(chunk or DEFAULT_CHUNK), shards.W)
        dev = edge_index.device
        self.device = dev
        N, U, NP, side = shards.N, shards.U, shards.NP, shards.side
        E = int(edge_index.shape[1])
        self.num_edges = E
        if E and (int(edge_index.min()) < 0 or int(edge_index.max()) >= N):
            raise IndexError(f"edge_index holds node ids outside [0, {N})")
        pm = torch.from_numpy(shards.padmap()).to(dev)
        eip = pm[edge_index]
        self.bipartite = bool(E == 0 or ((edge_index[0] < U) != (edge_index[1] < U)).all().item())
        stream = _ffi.stream_of(dev)
        owned = torch.from_numpy(shards.owned_mask(rank)).to(dev)
        # the whole graph's CSR over the padded ids (degrees, hence gcn_norm, of the whole graph);
        # only this rank's rows are scheduled
        self.fwd, self.dis, _ = _build_direction(eip[1].contiguous(), eip[0].contiguous(), NP, self.chunk, side, None,
                                                 stream, owned)
        del eip
        if self.bipartite:
            pieces = [("u", "i", torch.from_numpy(shards.owned_mask(rank, "i")).to(dev)),   # A: user sources
                      ("i", "u", torch.from_numpy(shards.owned_mask(rank, "u")).to(dev))]   # B: item sources
        else:
            pieces = [("ui", "ui", owned)]
        # the one-GPU plan's slicing decision and bounds at width slice_d
        # (lgcn_amd.plan.PropagationPlan.schedule), mapped to padded ids: the same segments, the
        # same hub chunks
        sd_ = int(slice_d or d)
        sb = slice_bytes_for(N, sd_)
        bounds = slice_bounds(N, U, sd_, sb) if (sb and E) else None
        if bounds is not None and not (E >= 8 * (len(bounds) - 1) * N or _slice_forced()):
            bounds = None
        self.halves: list[Half] = []
        # R > 1 (a rank holds a 1/R share of the rows): the plain item schedule, one launch per
        # half-layer, hub chunks of rank_chunk rows — a slice launch's fixed cost (its longest
        # chunk chain, ~10-25 us) outweighs the L2 locality it buys at that size
        # (profiles/r02k_shard/: per-rank K=3 step at 8x1 0.59 ms sliced, 0.25 ms plain)
        if shards.W > 1:
            bounds = None
        for reads, writes, mask in pieces:
            direction = None
            if bounds is not None:
                direction = build_sliced(self.fwd, NP, shards.pad_bounds(bounds), sliced_chunk(self.chunk), mask)
            if direction is None:
                f = self.fwd
                direction = CsrDirection(f.rowptr, f.col, f.eid, f.val,
                                         *_schedule(f.rowptr, NP, E, self.chunk, side, mask, stream), self.chunk)
            partial = (torch.empty((direction.n_partials, d), dtype=torch.float32, device=dev)
                       if direction.n_partials else None)
            self.halves.append(Half(direction, reads, writes, partial))
        # sliced: the running-sum buffers are needed (per-slice launches)
        self.sliced = bounds is not None and all(hasattr(h.direction, "launches") for h in self.halves)
        self.slice_bounds = bounds

    @property
    def NP(self) -> int:
        return self.shards.NP

    def run_half(self, h: Half, x: torch.Tensor, e: torch.Tensor | None, acc: torch.Tensor, y: torch.Tensor | None,
                 mode: int, div: float, mul: float) -> None:
        from .propagate import spmm

        NP = self.NP
        spmm(h.direction, NP, self.d, (x, None, NP), None if e is None else (e, None, NP), (acc, None, NP), y, mode,
             div, mul, h.partial)


def _slice_forced() -> bool:
    from . import tuning

    return tuning.get().slice_mb is not None


EXCHANGE_MODES = ("allgather", "p2p")


class BlockExchange:
    """all_gather of one block (every rank's user rows, or item rows) of a layer output.

    nccl (RCCL over xGMI), issued on a side stream after an event on the compute stream; the
    caller's stream waits on the returned event only before the half that reads the block:
    * ``allgather``: ``all_gather_into_tensor`` in place (each rank's chunk is its slice of the
      output block) — RCCL picks the algorithm (rings over the group);
    * ``p2p``: one send of this rank's chunk to every peer and one receive from every peer, as one
      ``batch_isend_irecv`` (a group of R ranks drives its R - 1 direct xGMI links at once).
    gloo (tests, rehearsal): the same exchange through host memory, synchronously."""

    def __init__(self, shards: RowShards, rank: int, group=None, members: list[int] | None = None,
                 mode: str = "allgather"):
        """rank: this rank's index among the ranks that share its columns (its RowShards rank);
        group: their process group (None = the default group); members: their global ranks in
        row-group order (p2p; default range(W)); mode: one of EXCHANGE_MODES."""
        import torch.distributed as dist

        if mode not in EXCHANGE_MODES:
            raise ValueError(f"exchange mode {mode!r} not in {EXCHANGE_MODES}")
        self.dist = dist
        self.shards, self.rank, self.group, self.mode = shards, rank, group, mode
        self.members = list(members) if members is not None else list(range(shards.W))
        if len(self.members) != shards.W:
            raise ValueError(f"{len(self.members)} exchange members for {shards.W} row groups")
        self.nccl = device_collectives(group)
        self.rccl = dist.is_initialized() and dist.get_backend(group) == "nccl"
        self.stream = None
        self.bytes = 0  # received per rank, over the run

    def _p2p_ops(self, out, mine, c):
        d = self.dist
        ops = []
        for p, peer in enumerate(self.members):
            if p != self.rank:
                ops.append(d.P2POp(d.isend, mine, peer, self.group))
                ops.append(d.P2POp(d.irecv, out[p * c:(p + 1) * c], peer, self.group))
        return ops

    def start(self, buf: torch.Tensor, b: str):
        lo, c = self.shards.block(b)
        W = self.shards.W
        out = buf[lo: lo + W * c]
        mine = out[self.rank * c:(self.rank + 1) * c]
        self.bytes += (W - 1) * c * buf.shape[1] * buf.element_size()
        if self.nccl:
            if self.stream is None:
                self.stream = torch.cuda.Stream(buf.device)
            ready = torch.cuda.Event()
            ready.record(torch.cuda.current_stream(buf.device))
            with torch.cuda.stream(self.stream):
                self.stream.wait_event(ready)
                if self.mode == "p2p":
                    if not self.rccl:
                        # gloo's send/recv move a device tensor's bytes from the host, outside
                        # every stream: the block must be final and its old readers done first
                        torch.cuda.synchronize(buf.device)
                    for req in self.dist.batch_isend_irecv(self._p2p_ops(out, mine, c)):
                        req.wait()
                else:
                    self.dist.all_gather_into_tensor(out, mine, group=self.group)
                done = torch.cuda.Event()
                done.record(self.stream)
            return done
        host = torch.empty((W * c, buf.shape[1]), dtype=buf.dtype)
        if self.mode == "p2p":
            host[self.rank * c:(self.rank + 1) * c] = mine.cpu()
            reqs = []
            for p, peer in enumerate(self.members):
                if p != self.rank:
                    reqs.append(self.dist.isend(host[self.rank * c:(self.rank + 1) * c], peer, group=self.group))
                    reqs.append(self.dist.irecv(host[p * c:(p + 1) * c], peer, group=self.group))
            for req in reqs:
                req.wait()
        else:
            self.dist.all_gather_into_tensor(host, mine.cpu().clone(), group=self.group)
        out.copy_(host)
        return None

    def wait(self, handle, device) -> None:
        if handle is not None:
            torch.cuda.current_stream(device).wait_event(handle)


def propagate_forward_sharded(x0p: torch.Tensor, splan, K: int, exchange: BlockExchange | None) -> torch.Tensor:
    """out[NP, d] = LightGCN final embedding of this rank's rows (padded ids; the other ranks' rows
    are not written). x0p: the whole padded layer-0 table (RowShards.to_padded), on every rank."""
    NP, d = x0p.shape
    if NP != splan.NP:
        raise ValueError(f"x0p has {NP} rows, the sharded plan {splan.NP}")
    dev = x0p.device
    out = torch.empty((NP, d), dtype=torch.float32, device=dev)
    div = float(K + 1)
    mul = float(np.float32(1.0 / (K + 1)))
    if K == 0:
        return (x0p / div) * mul
    bufs = [torch.empty((NP, d), dtype=torch.float32, device=dev) for _ in range(min(2, K - 1))]
    last_run = torch.empty((NP, d), dtype=torch.float32, device=dev) if splan.sliced else None
    pending: dict = {}
    for k in range(1, K + 1):
        src = x0p if k == 1 else bufs[(k - 2) % 2]
        dst = bufs[(k - 1) % 2] if k < K else None
        if K == 1:
            mode = _ffi.EPI_FINAL_E
        elif k == 1:
            mode = _ffi.EPI_INIT
        elif k < K:
            mode = _ffi.EPI_ADD
        else:
            mode = _ffi.EPI_FINAL_ACC
        final = mode in (_ffi.EPI_FINAL_E, _ffi.EPI_FINAL_ACC)
        e = x0p if mode in (_ffi.EPI_INIT, _ffi.EPI_FINAL_E) else None
        order = splan.halves if k % 2 == 1 else splan.halves[::-1]
        started: dict = {}
        for h in order:
            for b in h.reads:
                if b in pending:
                    exchange.wait(pending.pop(b), dev)
            # sliced schedules use y as the running row sums (the final layer's y is scratch: the
            # FINAL epilogues never write y)
            y = dst if dst is not None else last_run
            splan.run_half(h, src, e, out, y, mode, div if final else 1.0, mul if final else 1.0)
            if dst is not None and exchange is not None:
                for b in h.writes:
                    started[b] = exchange.start(dst, b)
        pending = started
    return out


# ---------------------------------------------------------------------------------------------
# "reduce" row groups: users sharded, item rows reduced (bipartite graphs)
# ---------------------------------------------------------------------------------------------
#
# The all_gather grid above moves every exchanged layer's whole output (users AND items, 57 MB per
# layer at C2 d = 64) to every rank of a column group. On a bipartite graph the item side is the
# small one (I = 59k of N = 222k at C2), and user rows only ever gather item rows. So:
#
# * row group g owns one edge-balanced range of USER rows; every rank holds every ITEM row;
# * user rows of layer k: the rank's own users, summed over all their in-edges (sources are items)
#   — the one-GPU plain schedule's rows, from the full item table of layer k-1;
# * item rows of layer k: each rank sums, for EVERY item, the in-edges whose source user it owns
#   (a CSR of that edge subset with the whole graph's gcn_norm weights); the R partial tables are
#   summed by one all_reduce per layer (RCCL, on a side stream, overlapped with the user pass);
#   the reduced rows of every layer are kept (the next user pass reads them anyway), and the
#   LightGCN layer-stack mean of the item rows runs once, at the end, on the rank's item share
#   (lgcn_stack_mean_rows: the INIT / ADD / FINAL_ACC epilogues' additions in their order).
# * "fused" (round 4): a layer's item-partial pass and user pass are independent (both read layer
#   k-1), so they can run as ONE launch (lgcn_spmm_pair) and their split-row combines as one more;
#   the layer's all_reduce then starts after both and the next layer waits for it (no overlap, one
#   launch gap and one drain per pair instead of two). Both orders are timed grid candidates.
#
# Exchange per rank per K-layer step: K all_reduces of I x d/F floats (a ring moves 2 (R-1)/R of
# it), instead of K-1 all_gathers of (R-1)/R of N x d/F. C2 at 8 x 1: 3 x 26.4 MB vs 2 x 52 MB;
# and a rank's item partials gather only its own 1/R of the user table (cache-resident).
# Numerics: a user row is one sequential chain as on one GPU; an item row is the sum of R partial
# chains (its users cut into R ranges), i.e. reassociated like a chunked hub row: within 1e-5.


@dataclasses.dataclass
class UserShards:
    """Edge-balanced user-row ranges of R row groups (items replicated)."""

    R: int
    U: int
    I: int
    ub: np.ndarray  # int64[R+1]

    @classmethod
    def build(cls, in_degree: np.ndarray, U: int, R: int) -> "UserShards":
        deg = np.asarray(in_degree, dtype=np.int64)
        if U < 0 or deg.size < U or R < 1:
            raise ValueError(f"bad shard request U={U} N={deg.size} R={R}")
        return cls(R, U, deg.size - U, balanced_bounds(deg[:U] + ROW_COST, R))

    @property
    def N(self) -> int:
        return self.U + self.I

    def users(self, g: int) -> tuple[int, int]:
        return int(self.ub[g]), int(self.ub[g + 1])


class ReducePlan:
    """Row group g's plans for the reduce mode (see above): its users' rows over the whole CSR and
    the item partials over the edges its users source."""

    def __init__(self, edge_index: torch.Tensor, shards: UserShards, g: int, d: int, chunk: int | None = None):
        from .plan import DEFAULT_CHUNK, CsrDirection, _build_direction, _schedule

        _ffi.require_device(edge_index, "ReducePlan")
        if edge_index.dim() != 2 or edge_index.shape[0] != 2 or edge_index.dtype != torch.int64:
            raise ValueError("edge_index must be int64 [2, E]")
        self.shards, self.g, self.d = shards, int(g), int(d)
        self.chunk = rank_chunk(int(chunk or DEFAULT_CHUNK), max(shards.R, 2))
        dev = edge_index.device
        N, U = shards.N, shards.U
        E = int(edge_index.shape[1])
        if E and (int(edge_index.min()) < 0 or int(edge_index.max()) >= N):
            raise IndexError(f"edge_index holds node ids outside [0, {N})")
        src, dst = edge_index[0].contiguous(), edge_index[1].contiguous()
        if E and not bool(((src < U) != (dst < U)).all().item()):
            raise ValueError("the reduce mode needs a bipartite user-item graph")
        stream = _ffi.stream_of(dev)
        ua, ub = shards.users(self.g)
        own = torch.zeros(N, dtype=torch.uint8, device=dev)
        own[ua:ub] = 1
        # the whole graph's CSR (its in-degrees give gcn_norm), scheduled on this group's users
        self.users, self.dis, bad = _build_direction(dst, src, N, self.chunk, U, None, stream, own)
        if bad:
            raise IndexError(f"edge_index holds {bad} edge(s) with a node id outside [0, {N})")
        self.users.block_split = False
        # the item partials: the edges whose source is one of this group's users, every item row
        # scheduled (0 where none), weights from the whole graph's degrees
        sel = (src >= ua) & (src < ub)
        items = torch.zeros(N, dtype=torch.uint8, device=dev)
        items[U:] = 1
        self.partial, _, _ = _build_direction(dst[sel].contiguous(), src[sel].contiguous(), N, self.chunk, U,
                                              self.dis, stream, items)
        self.partial.block_split = False
        # the pair combine (fused order) packs the thousands of 2-16-chunk split rows by lane group
        from .plan import pack_split_rows

        pack_split_rows(self.users)
        pack_split_rows(self.partial)
        # the last layer's item rows are reduce-scattered: this group's share of the items
        # (I padded to a multiple of R; padding rows are zero partials that no pass writes)
        R = shards.R
        self.I_pad = -(-shards.I // R) * R
        per = self.I_pad // R
        self.share = (min(shards.I, self.g * per), min(shards.I, (self.g + 1) * per))
        self.n_sub = int(sel.sum().item())
        self.scratch = {}

    def item_tables(self, K: int, I_pad: int, d: int, dev) -> list:
        """K zeroed [I_pad, d] item tables of propagate_forward_reduced, allocated once per (K, d).
        Only the padding rows' zeros are relied on: every pass writes rows [0, I)."""
        key = ("items", K, I_pad, d)
        if key not in self.scratch:
            self.scratch[key] = [torch.zeros((I_pad, d), dtype=torch.float32, device=dev) for _ in range(K)]
        return self.scratch[key]

    def _part(self, direction, d):
        key = (id(direction), d)
        if direction.n_partials and key not in self.scratch:
            self.scratch[key] = torch.empty((direction.n_partials, d), dtype=torch.float32,
                                            device=direction.rowptr.device)
        return self.scratch.get(key)

    # the three kinds of pass; tables are (lo, hi, split = U) split tables
    def _pass(self, direction, x, e, y, acc, mode: int, div: float, mul: float):
        """direction's lgcn_pass_t (its split rows combined packed: pack_split_rows' n_split_big)."""
        N, d = self.shards.N, self.d
        el, eh, es = e if e is not None else (None, None, N)
        return _ffi.Pass(direction.items.data_ptr(), direction.n_items, direction.splits.data_ptr(),
                         direction.n_splits, direction.col.data_ptr(), direction.val.data_ptr(),
                         _ffi.ptr(x[0]), _ffi.ptr(x[1]), x[2], _ffi.ptr(el), _ffi.ptr(eh), es, _ffi.ptr(y),
                         _ffi.ptr(acc[0]), _ffi.ptr(acc[1]), acc[2], _ffi.ptr(self._part(direction, d)), mode, div,
                         mul, n_split_big=getattr(direction, "n_split_big", -1))

    def _run(self, p, dev) -> None:
        import contextlib
        import ctypes

        from . import propagate

        timer = propagate._launch_timer  # bench.py's launch brackets (one pass: items + combine)
        with (timer(self.d, 1) if timer is not None else contextlib.nullcontext()):
            _ffi.check(_ffi.load().lgcn_spmm_pass(ctypes.byref(p), self.shards.N, self.d, 3, _ffi.stream_of(dev)),
                       "lgcn_spmm_pass")

    def run_partial(self, x_users: torch.Tensor, part_items: torch.Tensor) -> None:
        U = self.shards.U
        self._run(self._pass(self.partial, (x_users, part_items, U), None, None, (part_items, part_items, U),
                             _ffi.EPI_STORE, 1.0, 1.0), x_users.device)

    def run_users(self, x_items: torch.Tensor, e, acc, y, mode: int, div: float, mul: float) -> None:
        U = self.shards.U
        self._run(self._pass(self.users, (x_items, x_items, U), e, y, acc, mode, div, mul), x_items.device)

    def run_pair(self, x_users: torch.Tensor, part_items: torch.Tensor, x_items: torch.Tensor, e, acc, y, mode: int,
                 div: float, mul: float) -> None:
        """run_partial and run_users of one layer as two launches (lgcn_spmm_pair: both item passes
        in one, both combines in the other) — the same per-row arithmetic."""
        import ctypes

        U = self.shards.U
        pa = self._pass(self.partial, (x_users, part_items, U), None, None, (part_items, part_items, U),
                        _ffi.EPI_STORE, 1.0, 1.0)
        pb = self._pass(self.users, (x_items, x_items, U), e, y, acc, mode, div, mul)
        import contextlib

        from . import propagate

        timer = propagate._launch_timer  # one bracket over both passes: counted as their two launches
        with (timer(self.d, 2) if timer is not None else contextlib.nullcontext()):
            _ffi.check(_ffi.load().lgcn_spmm_pair(ctypes.byref(pa), ctypes.byref(pb), self.shards.N, self.d, 3,
                                                  _ffi.stream_of(x_users.device)), "lgcn_spmm_pair")

    def finish_items(self, x0i: torch.Tensor, layers: list, last_share: torch.Tensor, out_i: torch.Tensor,
                     div: float, mul: float) -> None:
        """out_i[a:b] = the layer-stack mean of this group's item share [a, b): x0i, the reduced rows
        of layers 1..K-1 (layers, all items) and layer K's share (last_share, row a at row 0)."""
        a, b = self.share
        if b <= a:
            return
        import ctypes

        ys = [t[a:b] for t in layers] + [last_share[:b - a]]
        arr = (ctypes.c_void_p * len(ys))(*[t.data_ptr() for t in ys])
        _ffi.check(_ffi.load().lgcn_stack_mean_rows(x0i[a:b].data_ptr(), arr, len(ys), b - a, self.d,
                                                    out_i[a:b].data_ptr(), div, mul,
                                                    _ffi.stream_of(x0i.device)), "lgcn_stack_mean_rows")


class ItemReducer:
    """Sum of the R item-partial tables of a column group: one all_reduce per layer (nccl: RCCL on
    a side stream after an event on the compute stream, waited on before the rows are read; gloo:
    synchronous, through host memory).

    method "a2a" (round 5) replaces RCCL's all_reduce by its two halves written out: one
    all_to_all_single sends slice s of the rank's partial table to group rank s (on a fully
    connected xGMI mesh every pair has its own link, so the R - 1 transfers run at once instead of
    around a ring), the owner sums the R slices it received in rank order (lgcn_stack_mean_rows with
    div = mul = 1: ((p_0 + p_1) + ...) exactly), and one all_gather_into_tensor returns the reduced
    slices to every rank; the last layer stops after the sum (its reduce_scatter). Same bytes as a
    ring all_reduce, other latency and link use: bench.py times both (reduce-a2a candidates)."""

    def __init__(self, R: int, group=None, method: str = "ring"):
        import torch.distributed as dist

        if method not in ("ring", "a2a"):
            raise ValueError(f"ItemReducer method {method!r}: 'ring' or 'a2a'")
        self.dist, self.R, self.group, self.method = dist, int(R), group, method
        self.nccl = R > 1 and device_collectives(group)
        self.stream = None
        self.ws = {}
        self.bytes = 0  # ring all_reduce traffic received per rank over the run

    def _a2a(self, buf: torch.Tensor, out_share: torch.Tensor | None, rank: int):
        """The a2a method's reduce: rank `rank` of the group sums slice `rank` of the R partial
        tables in rank order into out_share (or, None, a workspace all-gathered back into buf)."""
        R, dist = self.R, self.dist
        per = buf.shape[0] // R
        if not self.nccl:  # gloo through host memory: the same slices, sums and order
            host = buf.cpu()
            recv = torch.empty_like(host)
            dist.all_to_all_single(recv, host, group=self.group)
            acc = recv[:per].clone()
            for s in range(1, R):
                acc += recv[s * per:(s + 1) * per]
            if out_share is not None:
                out_share.copy_(acc)
                return None
            parts = [torch.empty_like(acc) for _ in range(R)]
            dist.all_gather(parts, acc, group=self.group)
            buf.copy_(torch.cat(parts))
            return None
        import ctypes

        key = (tuple(buf.shape), buf.device)
        if key not in self.ws:
            self.ws[key] = (torch.empty_like(buf), torch.empty((per, buf.shape[1]), dtype=buf.dtype, device=buf.device))
        recv, mine = self.ws[key]
        dst = out_share if out_share is not None else mine
        if self.stream is None:
            self.stream = torch.cuda.Stream(buf.device)
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(buf.device))
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(ready)
            dist.all_to_all_single(recv, buf, group=self.group)
            ys = (ctypes.c_void_p * (R - 1))(*[recv[s * per:(s + 1) * per].data_ptr() for s in range(1, R)])
            _ffi.check(_ffi.load().lgcn_stack_mean_rows(recv[:per].data_ptr(), ys, R - 1, per, buf.shape[1],
                                                        dst.data_ptr(), 1.0, 1.0, _ffi.stream_of(buf.device)),
                       "lgcn_stack_mean_rows (a2a slice sum)")
            if out_share is None:
                dist.all_gather_into_tensor(buf, mine, group=self.group)
            done = torch.cuda.Event()
            done.record(self.stream)
        return done

    def start_scatter(self, buf: torch.Tensor, out: torch.Tensor, rank: int):
        """out = this group member's 1/R row share of the sum of buf over the group (buf's rows a
        multiple of R): reduce_scatter (nccl), or through host memory (gloo)."""
        self.bytes += int((self.R - 1) / self.R * buf.numel() * buf.element_size())
        if self.R == 1:
            out.copy_(buf)
            return None
        if self.method == "a2a":
            return self._a2a(buf, out, rank)
        if self.nccl:
            if self.stream is None:
                self.stream = torch.cuda.Stream(buf.device)
            ready = torch.cuda.Event()
            ready.record(torch.cuda.current_stream(buf.device))
            with torch.cuda.stream(self.stream):
                self.stream.wait_event(ready)
                self.dist.reduce_scatter_tensor(out, buf, op=self.dist.ReduceOp.SUM, group=self.group)
                done = torch.cuda.Event()
                done.record(self.stream)
            return done
        host = buf.cpu()
        self.dist.all_reduce(host, op=self.dist.ReduceOp.SUM, group=self.group)
        per = buf.shape[0] // self.R
        out.copy_(host[rank * per:(rank + 1) * per])
        return None

    def start(self, buf: torch.Tensor):
        self.bytes += int(2 * (self.R - 1) / self.R * buf.numel() * buf.element_size())
        if self.R == 1:
            return None
        if self.method == "a2a":
            return self._a2a(buf, None, self.dist.get_rank(self.group))
        if self.nccl:
            if self.stream is None:
                self.stream = torch.cuda.Stream(buf.device)
            ready = torch.cuda.Event()
            ready.record(torch.cuda.current_stream(buf.device))
            with torch.cuda.stream(self.stream):
                self.stream.wait_event(ready)
                self.dist.all_reduce(buf, op=self.dist.ReduceOp.SUM, group=self.group)
                done = torch.cuda.Event()
                done.record(self.stream)
            return done
        host = buf.cpu()
        self.dist.all_reduce(host, op=self.dist.ReduceOp.SUM, group=self.group)
        buf.copy_(host)
        return None

    def wait(self, handle, device) -> None:
        if handle is not None:
            torch.cuda.current_stream(device).wait_event(handle)


def propagate_forward_reduced(x0u: torch.Tensor, x0i: torch.Tensor, rplan, K: int,
                              reducer: ItemReducer, fused: bool = False) -> tuple[torch.Tensor, torch.Tensor]:
    """(users [U, d], items [I, d]): the LightGCN final embedding of this row group's users and of
    its share of the items, rplan.share = [a, b) (other rows unwritten). x0u / x0i: the layer-0
    tables (this rank's columns).

    Layer k: the item partials from the users of layer k-1 (own rows), their all_reduce started;
    then, once layer k-1's reduction has landed, the users of layer k from the items of layer k-1.
    Each reduction overlaps a user pass. fused=True runs a layer's two passes as one pair of
    launches (lgcn_spmm_pair) and starts its reduction after them. The last layer's partials are
    reduce-scattered (each group member gets its share of the items: half a ring all_reduce's
    bytes); the reduced rows of every layer are kept, and the item rows' layer-stack mean runs once
    on the share (rplan.finish_items)."""
    U, d = x0u.shape
    I = x0i.shape[0]
    dev = x0u.device
    div = float(K + 1)
    mul = float(np.float32(1.0 / (K + 1)))
    out_u = torch.empty((U, d), dtype=torch.float32, device=dev)
    out_i = torch.empty((I, d), dtype=torch.float32, device=dev)
    if K == 0:
        return (x0u / div) * mul, (x0i / div) * mul
    yu = [torch.empty((U, d), dtype=torch.float32, device=dev) for _ in range(min(2, K - 1))]
    I_pad = getattr(rplan, "I_pad", I)
    # the reduced item rows of layers 1..K-1 (read by the next user pass and by the final mean),
    # and layer K's partials (reduce-scattered into `share`); padding rows stay zero. Every pass
    # writes every item row (rows without a partial edge get a zero-length item), so the tables are
    # allocated zeroed once per plan and reused (no fill kernels per step)
    bufs = getattr(rplan, "item_tables", None)
    part = bufs(K, I_pad, d, dev) if bufs is not None else \
        [torch.zeros((I_pad, d), dtype=torch.float32, device=dev) for _ in range(K)]
    share = torch.empty((I_pad // max(1, reducer.R), d), dtype=torch.float32, device=dev)
    e = (x0u, x0i, U)
    acc = (out_u, out_i, U)

    def mode_of(k):
        if K == 1:
            return _ffi.EPI_FINAL_E
        return _ffi.EPI_INIT if k == 1 else (_ffi.EPI_ADD if k < K else _ffi.EPI_FINAL_ACC)

    def start(k):
        if k < K:
            return reducer.start(part[k - 1])
        return reducer.start_scatter(part[k - 1], share, rplan.g)  # the last layer: this member's share

    pending = None  # the reduction in flight
    for k in range(1, K + 1):
        src_u = x0u if k == 1 else yu[(k - 2) % 2]
        src_i = x0i if k == 1 else part[k - 2]
        mode = mode_of(k)
        final = mode in (_ffi.EPI_FINAL_E, _ffi.EPI_FINAL_ACC)
        y = yu[(k - 1) % 2] if k < K else None
        ue = e if mode in (_ffi.EPI_INIT, _ffi.EPI_FINAL_E) else None
        udiv, umul = (div, mul) if final else (1.0, 1.0)
        if fused:
            reducer.wait(pending, dev)  # layer k-1's items: reduced before this layer's users read them
            rplan.run_pair(src_u, part[k - 1], src_i, ue, acc, y, mode, udiv, umul)
            pending = start(k)
        else:
            rplan.run_partial(src_u, part[k - 1])
            started = start(k)
            reducer.wait(pending, dev)
            rplan.run_users(src_i, ue, acc, y, mode, udiv, umul)
            pending = started
    reducer.wait(pending, dev)
    rplan.finish_items(x0i, part[:K - 1], share, out_i, div, mul)
    return out_u, out_i
