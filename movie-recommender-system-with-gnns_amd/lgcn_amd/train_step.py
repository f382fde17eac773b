"""The Cluster-GCN training step without autograd: the reference's per-batch step
(reference utils/train_test.py:86-101: zero_grad, compute_embeddings, bpr_loss, backward,
clip_grad_norm_(1), Adam step) as a fixed sequence of HIP launches.

    out  = LightGCN forward over the batch edges       (lgcn_spmm x K over a touched-only plan)
    neg  = torch.randint(0, I, (B,))                   (same draw as reference sample_negative;
                                                        eager before a graph replay)
    loss, per-triplet grad rows = lgcn_bpr_fused       (+ lgcn_bpr_loss)
    g    = scaled dF rows in a fixed order, written    (lgcn_csr_build over the 3B keys +
           straight into the two gradient tables        lgcn_segment_rows with the backward scale)
    grads = LightGCN backward seeded with g, in place (lgcn_spmm x K, transposed touched-only plan)
          + reg-gradient rows                          (lgcn_segment_rows, add)
    [all_reduce grads over ranks]; FusedAdam (clip fused) or any torch optimizer

Sparse batch (exact): a Cluster-GCN batch's edges touch a few % of the N rows. Its plans schedule
only those rows. A row no batch edge reaches gets an exact 0 from every layer, so its final
embedding is (x0 / (K+1)) * fp32(1/(K+1)) — lgcn_bpr_fused computes that on the fly for
negatives that land there — and its gradient is just the seed g. So no full-N epilogue runs;
the only dense passes left are the gradient-table write and the optimizer.

Per batch the (user, positive) triplet halves are a fixed function of the batch edges
(reference utils/helpers.py:98-99), so they are computed once and cached with the plan; only the
negatives are drawn each step. No host synchronisation happens inside a step.
"""
from __future__ import annotations


import torch

from . import _ffi
import numpy as np

from .propagate import propagate_backward_seeded, propagate_forward, spmm


class ColumnGroup:
    """This rank's share of column-sharded training (SURVEY §8e's parity-preserving alternative to
    data parallelism): W ranks train the SAME batch with the same negatives, rank r holding columns
    [r*d/W, (r+1)*d/W) of both tables and their Adam state. LightGCN never mixes columns, so the
    propagation and the row-wise Adam need nothing from the other ranks; the cosine-BPR loss needs
    each triplet's full-width dot products and norms (one all_reduce of [B, 6] per step) and
    clip_grad_norm_ the full norm (one all_gather of the norm's block partials). The result is the
    one-GPU step up to the association of those sums (reference utils/train_test.py:18-51,86-96)."""

    def __init__(self, world: int, rank: int, d_full: int, group=None):
        if d_full % world or (d_full // world) % 4:
            raise ValueError(f"d={d_full} does not split into {world} column shares of a multiple of 4")
        self.world, self.rank, self.d_full, self.group = int(world), int(rank), int(d_full), group
        self.d = self.d_full // self.world
        self._gathered = None  # every rank's norm partials (persistent: graph replays write it)
        self.capture = None    # a _SegmentedGraph while a step is being captured

    @property
    def cols(self) -> tuple[int, int]:
        return self.rank * self.d, (self.rank + 1) * self.d

    def _all_reduce(self, t: torch.Tensor) -> None:
        import torch.distributed as dist

        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)

    def all_reduce(self, t: torch.Tensor) -> None:
        """t (this rank's [B, 6] partial sums) summed over the column groups, in place. While a
        step is being captured, the capture is cut here and the all_reduce runs eagerly between
        the graphs at replay."""
        if self.world == 1:
            return
        if self.capture is not None:
            self.capture.split(lambda: self._all_reduce(t))
            return
        self._all_reduce(t)

    def _gather(self, out: torch.Tensor, part: torch.Tensor) -> None:
        import torch.distributed as dist

        from .distributed import device_collectives

        if device_collectives(self.group):
            dist.all_gather_into_tensor(out, part, group=self.group)
        else:
            dist.all_gather(list(out.view(self.world, -1).unbind(0)), part, group=self.group)

    def gather_partials(self, part: torch.Tensor) -> torch.Tensor:
        """Every rank's norm partials in rank order (cut point of a capture, as all_reduce)."""
        if self.world == 1:
            return part
        if self._gathered is None or self._gathered.numel() != self.world * part.numel():
            if self.capture is not None:
                raise RuntimeError("ColumnGroup: take one eager step before capturing (norm partials buffer)")
            self._gathered = torch.empty(self.world * part.numel(), dtype=part.dtype, device=part.device)
        out = self._gathered
        if self.capture is not None:
            self.capture.split(lambda: self._gather(out, part))
        else:
            self._gather(out, part)
        return out

    def reg_coeff(self, coeff: float) -> float:
        """The coefficient whose kreg = c * 2 / (B * d) over this rank's d columns equals the full
        width's coeff * 2 / (B * d_full) (the reg rows the scatters form, RegSrc)."""
        return float(np.float32(float(coeff) * self.d / self.d_full))


class _SegmentedGraph:
    """A training step captured as hipGraphs cut at its eager collectives (column-sharded
    training: the [B, 6] all_reduce and the norm partials' all_gather): replay() runs graph 0,
    collective 0, graph 1, ... in capture order. The graphs share one private memory pool, which
    is safe because they always replay in the order they were captured."""

    def __init__(self):
        self.graphs, self.colls = [], []
        self.pool = torch.cuda.graph_pool_handle()
        self.program = _programs_on()  # each segment issued as a launch program (StepProgram)

    def _begin(self) -> None:
        g = _new_graph(self.program)
        g.capture_begin(pool=self.pool)
        self.graphs.append(g)

    def split(self, collective) -> None:
        self.graphs[-1].capture_end()
        self.colls.append(collective)
        self._begin()

    def capture(self, fn):
        torch.cuda.synchronize()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            self._begin()
            try:
                out = fn()
            finally:
                self.graphs[-1].capture_end()
        torch.cuda.current_stream().wait_stream(side)
        self.graphs = [_replayable(g, self.program) for g in self.graphs]
        return out

    def replay(self) -> None:
        for i, g in enumerate(self.graphs):
            g.replay()
            if i < len(self.colls):
                self.colls[i]()


class StepProgram:
    """A captured step issued as plain launches on the current stream (lgcn_program_run, ABI 11)
    instead of a hipGraph replay: the graph's kernels, memsets and copies, read once from the
    captured graph, launched from one C call. Measured (tools/train_eager_pair.sh,
    profiles/r06zf_eager/): a hipGraph replay costs the GPU ~8 us of its own per step (the eager
    step's kernels run back to back: C3 0.143 vs 0.151 ms, planted 0.445 vs 0.451 ms), but the
    eager step's Python issue takes 0.130 ms — nearly the step. The program issues the captured
    launches with neither cost. `graph` is a torch.cuda.CUDAGraph(keep_graph=True) after capture:
    it is kept (its nodes own the argument buffers, its pool the step's buffers) and only replayed
    as a graph if the library refuses it (a node with no stream-launch form)."""

    def __init__(self, graph):
        import ctypes

        self.graph = graph
        self._h = None
        lib = _ffi.load()
        h = ctypes.c_void_p()
        rc = lib.lgcn_program_from_graph(graph.raw_cuda_graph(), ctypes.byref(h))
        if rc == _ffi.E_UNSUPPORTED:
            self.refused = lib.lgcn_last_error().decode(errors="replace")
            self.launches = None
            return
        _ffi.check(rc, "lgcn_program_from_graph")
        self.refused = None
        self._h = h.value
        self.launches = int(lib.lgcn_program_launches(self._h))

    def replay(self) -> None:
        if self._h is None:
            self.graph.replay()
            return
        _ffi.check(_ffi.load().lgcn_program_run(self._h, torch.cuda.current_stream().cuda_stream),
                   "lgcn_program_run")

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        try:
            if h is not None and _ffi._lib is not None:
                _ffi._lib.lgcn_program_free(h)
        except Exception:  # interpreter shutdown: the module may already be torn down
            pass


def _programs_on() -> bool:
    from . import tuning

    return tuning.get().step_program


def _new_graph(program: bool):
    """A CUDAGraph to capture into: kept after capture (not instantiated) when it will be issued as
    a launch program (StepProgram needs the graph's nodes)."""
    return torch.cuda.CUDAGraph(keep_graph=True) if program else torch.cuda.CUDAGraph()


def _replayable(g, program: bool):
    return StepProgram(g) if program else g


def batch_chunk_for(edges: int) -> int:
    """Hub chunk of a batch's propagation plan (edges: the batch's directed edges) and of its fixed
    gradient rows' segment plans (edges: their 2B contributions). Short chunks while the batch is small (its item
    passes are latency chains: more, shorter chains), longer ones for the big intra-part batches of
    a structured graph (fewer partials and block-split chains). Measured, K=3, d=128 (ms per step,
    profiles/r05y_batch_chunk/): 20k edges 0.162 / 0.163 / 0.177 at 16 / 32 / 64; 80-90k edges
    0.385 / 0.395 / 0.418 and 0.340 / 0.347 / 0.381 at 32 / 64 / 128; 360k edges 0.489 / 0.464 /
    0.456 / 0.456 / 0.459 at 32 / 64 / 128 / 256 / 512. lgcn_amd.tuning's batch_chunk forces one."""
    from . import tuning

    forced = tuning.get().batch_chunk
    if forced is not None:
        return int(forced)
    if edges >= 240_000:
        return 128
    if edges >= 160_000:
        return 64
    return 32


class _BatchState:
    def __init__(self, model, edge_index: torch.Tensor, d: int, lazy: bool = False):
        dev = edge_index.device
        U, I = model.num_users, model.num_items
        N = U + I
        from .plan import PropagationPlan

        self.plan = PropagationPlan(edge_index, N, batch_chunk_for(int(edge_index.shape[1])), side_split=U,
                                    touched_only=True)
        src, dst = edge_index[0], edge_index[1]
        self.users = src[src < U].contiguous()
        self.pos = (dst[dst >= U] - U).contiguous()
        if self.users.numel() != self.pos.numel():
            raise ValueError("batch is not a symmetric bipartite edge list: users and positives differ in count")
        B = self.B = int(self.users.numel())
        self.n_edges = int(edge_index.shape[1])  # the harness's loss weight (reference :101)
        self.neg = torch.empty(B, dtype=torch.int64, device=dev)
        self.keys = torch.empty(3 * B, dtype=torch.int64, device=dev)
        self.keys[:B] = self.users
        self.keys[B:2 * B] = self.pos + U
        # fixed (user, positive) gradient rows: load-balanced segment plans, built once per batch
        from .plan import segment_directions

        # fixed segment plans + range scatter (any batch whose 3B contribution ids fit int32; the
        # plans are built over max(N, 2B) rows, so batches with 2B > N — structured graphs, where
        # most edges stay intra-part — take this path too); else one sort of all keys per step
        self.small = 3 * B < 2**31
        self.lazy = lazy and self.small
        if self.lazy:
            # row-lazy optimizer: only the batch's touched rows (and the negatives) are written
            self.fixed_dense, self.fixed_sparse, self.fixed_touched = segment_directions(
                self.keys[:2 * B], N, chunk=batch_chunk_for(2 * B), row_mask=self.plan.touched)
            self.touched_rows = torch.nonzero(self.plan.touched).squeeze(1).to(torch.int32).contiguous()
            # ascending: the user rows first (HybridExchange packs only those)
            self.touched_users = self.touched_rows[:int((self.touched_rows < U).sum())]
        elif self.small:
            self.fixed_dense, self.fixed_sparse = segment_directions(self.keys[:2 * B], N, chunk=batch_chunk_for(2 * B))
        if self.small and B >= sorted_scatter_min_b():
            # large B: the negatives are grouped by row once per step and scattered row by row
            # (lgcn_sorted_scatter_add); the grouping is a counting sort (lgcn_group_keys) or,
            # with LGCN_NEG_GROUPING=radix, one stable radix sort (lgcn_csr_build over the B keys)
            # — the same rowptr / perm either way
            self.neg_rowptr = torch.empty(I + 1, dtype=torch.int64, device=dev)
            self.neg_perm = torch.empty(B, dtype=torch.int32, device=dev)
            self.neg_err = torch.zeros(1, dtype=torch.int64, device=dev)
            self.neg_grouping = neg_grouping()
            if self.neg_grouping == "radix":
                self.neg_col = torch.empty(B, dtype=torch.int32, device=dev)
                lib_ = _ffi.load()
                nb = _ffi._sz(0)
                _ffi.check(lib_.lgcn_csr_workspace_size(B, I, nb), "lgcn_csr_workspace_size")
                self.neg_ws = torch.empty(max(1, nb.value), dtype=torch.uint8, device=dev)
            else:
                # all zero between calls (lgcn_group_keys leaves it zeroed)
                n_cur = int(_ffi.load().lgcn_group_keys_cursor_len(max(1, I)))
                self.neg_cursor = torch.zeros(n_cur, dtype=torch.int32, device=dev)
        else:
            self.neg_rowptr = None
        if self.small:
            # the rows holding (user, positive) keys: lgcn_reg_rows_add visits only these
            rp = self.fixed_sparse.rowptr
            self.reg_rows = torch.nonzero(rp[1:] > rp[:-1]).squeeze(1).to(torch.int32).contiguous()
            # the range scatter parks each negative row's reg sum here; the sorted path forms them
            # after the backward instead (add_negative_reg_rows), so it needs no [B, d] table
            self.c2buf = torch.empty((B if self.neg_rowptr is None else 1, d), dtype=torch.float32, device=dev)
            self.c2flag = torch.empty(B, dtype=torch.uint8, device=dev)
            self.overflow = torch.zeros(1, dtype=torch.int32, device=dev)
            # the range scatter's per-row key counts when the reg rows are formed in the update
            # (lgcn_range_scatter_add_counts; the sorted path counts by neg_rowptr)
            self.neg_count = torch.empty(max(1, I), dtype=torch.int32, device=dev) if self.neg_rowptr is None else None
        self.cf = torch.empty((3 * B, d), dtype=torch.float32, device=dev)
        # reg-gradient rows: materialised only for the large-batch sort path; the segment-plan path
        # forms their sums from the layer-0 rows (lgcn_reg_rows_add, the scatters' reg source)
        self.cw = None if self.small else torch.empty((3 * B, d), dtype=torch.float32, device=dev)
        self.terms = torch.empty(2 * B, dtype=torch.float32, device=dev)
        self.loss = torch.empty(1, dtype=torch.float32, device=dev)
        self.loss_part = torch.empty(2 * _ffi.LOSS_PARTS, dtype=torch.float32, device=dev)
        self.rowptr = torch.empty(N + 1, dtype=torch.int64, device=dev)
        self.col = torch.empty(3 * B, dtype=torch.int32, device=dev)
        self.eid = torch.empty(3 * B, dtype=torch.int32, device=dev)
        self.err = torch.zeros(1, dtype=torch.int64, device=dev)
        lib = _ffi.load()
        nbytes = _ffi._sz(0)
        _ffi.check(lib.lgcn_csr_workspace_size(3 * B, N, nbytes), "lgcn_csr_workspace_size")
        self.ws = torch.empty(max(1, nbytes.value), dtype=torch.uint8, device=dev)
        self.plan.bwd  # build the transposed plan now (its build reads counts back once)


def neg_grouping() -> str:
    """How the sorted negatives path groups the B keys by row: "count" (lgcn_group_keys, the
    default) or "radix" (lgcn_csr_build); lgcn_amd.tuning's neg_grouping."""
    from . import tuning

    return tuning.get().neg_grouping


def sorted_scatter_min_b() -> int:
    """Batch size from which the negatives go through the sorted scatter instead of the range
    scatter (whose key streaming grows as B^2): measured on the C3 graphs (B ~ 1e4: range
    scatter ~10 us; B ~ 1.6e5: 627 us range vs sort + scatter). lgcn_amd.tuning's sorted_scatter_min_b."""
    from . import tuning

    return tuning.get().sorted_scatter_min_b


def loss_fused(st, I: int, cols=None) -> bool:
    """Whether the step's loss sum rides in the range scatter's launch (lgcn_range_scatter_add_loss:
    one extra workgroup, the same single-block sum as lgcn_bpr_loss) instead of its own launch:
    the range-scatter path, a batch small enough for the single-block sum, full-width rows."""
    return cols is None and st.neg_rowptr is None and I > 0 and 1 <= st.B < _ffi.LOSS_FUSED_MAX_B


def scatter_negatives(lib, st, gu, gi, U: int, I: int, d: int, mul: float, div: float, store_unless, stream,
                      uw, iw, coeff: float, loss=None, counts: bool = False, loss_acc=None) -> None:
    """dF rows of the step's negatives into the gradient tables and the first-occurrence flags
    (st.c2flag); the range scatter also parks each row's reg-rows sum (formed from the layer-0
    rows uw / iw) in its first-occurrence slot for add_negative_reg_rows after the backward — or,
    counts=True (the reg rows formed in the update), writes each row's key count to st.neg_count.
    loss = (terms, d, coeff, out): the step's loss sum in the same launch (loss_fused); loss_acc =
    (acc, w) with counts and loss: acc[0] += double(loss) * w there too (the harness's epoch sum)."""
    B = st.B
    C = st.cf[2 * B:]
    reg = (None, uw.data_ptr(), iw.data_ptr(), U, coeff, B)
    if st.neg_rowptr is None and counts:
        terms, ld, lcoeff, out = loss if loss is not None else (None, 0, 0.0, None)
        acc, w = loss_acc if loss_acc is not None else (None, 0.0)
        _ffi.check(lib.lgcn_range_scatter_add_counts(st.neg.data_ptr(), B, I, U, C.data_ptr(), d, gu.data_ptr(),
                                                     gi.data_ptr(), U, mul, div, st.c2flag.data_ptr(),
                                                     st.overflow.data_ptr(), _ffi.ptr(store_unless),
                                                     st.neg_count.data_ptr(), _ffi.ptr(terms),
                                                     B if terms is not None else 0, ld, lcoeff, _ffi.ptr(out),
                                                     _ffi.ptr(acc), float(w), stream),
                   "lgcn_range_scatter_add_counts")
        return
    if loss_acc is not None:
        raise ValueError("scatter_negatives: loss_acc needs the counted range scatter with the fused loss")
    if st.neg_rowptr is None:
        common = (st.neg.data_ptr(), B, I, U, C.data_ptr(), d, gu.data_ptr(), gi.data_ptr(), U, mul, div, *reg,
                  st.c2buf.data_ptr(), st.c2flag.data_ptr(), st.overflow.data_ptr(), _ffi.ptr(store_unless))
        if loss is not None:
            terms, ld, lcoeff, out = loss
            _ffi.check(lib.lgcn_range_scatter_add_loss(*common, terms.data_ptr(), B, ld, lcoeff, out.data_ptr(),
                                                       stream), "lgcn_range_scatter_add_loss")
        else:
            _ffi.check(lib.lgcn_range_scatter_add(*common, stream), "lgcn_range_scatter_add")
        return
    if loss is not None:
        raise ValueError("scatter_negatives: the fused loss needs the range-scatter path")
    if st.neg_grouping == "radix":
        _ffi.check(lib.lgcn_csr_build(st.neg.data_ptr(), st.neg.data_ptr(), B, I, st.neg_rowptr.data_ptr(),
                                      st.neg_col.data_ptr(), st.neg_perm.data_ptr(), st.neg_err.data_ptr(),
                                      st.neg_ws.data_ptr(), st.neg_ws.numel(), stream), "lgcn_csr_build(negatives)")
    else:
        _ffi.check(lib.lgcn_group_keys(st.neg.data_ptr(), B, I, st.neg_rowptr.data_ptr(), st.neg_perm.data_ptr(),
                                       st.neg_cursor.data_ptr(), st.neg_err.data_ptr(), stream),
                   "lgcn_group_keys(negatives)")
    # sorted path: no parked reg sums (add_negative_reg_rows forms them per row after the backward);
    # the first-occurrence flags are still written
    _ffi.check(lib.lgcn_sorted_scatter_add(st.neg_rowptr.data_ptr(), st.neg_perm.data_ptr(), I, U, C.data_ptr(), d,
                                           gu.data_ptr(), gi.data_ptr(), U, mul, div, None, None, None, 0, 0.0, 0,
                                           st.c2buf.data_ptr(), st.c2flag.data_ptr(), _ffi.ptr(store_unless), stream),
               "lgcn_sorted_scatter_add")


def add_negative_reg_rows(lib, st, gu, gi, U: int, d: int, uw, iw, coeff: float, stream) -> None:
    """The negatives' reg-gradient rows, after the backward: the range scatter's parked per-row sums
    (lgcn_flagged_rows_add), or — sorted path — the same n-copies sums formed per grouped row
    (lgcn_grouped_reg_add: no [B, d] parking table written and read back)."""
    if st.neg_rowptr is None:
        _ffi.check(lib.lgcn_flagged_rows_add(st.neg.data_ptr(), st.B, U, st.c2buf.data_ptr(), st.c2flag.data_ptr(), d,
                                             gu.data_ptr(), gi.data_ptr(), U, stream), "lgcn_flagged_rows_add")
        return
    _ffi.check(lib.lgcn_grouped_reg_add(st.neg_rowptr.data_ptr(), st.neg_rowptr.numel() - 1, U, uw.data_ptr(),
                                        iw.data_ptr(), U, d, coeff, st.B, gu.data_ptr(), gi.data_ptr(), U, stream),
               "lgcn_grouped_reg_add")


def add_fixed_reg_rows(lib, st, gu, gi, U: int, N: int, d: int, uw, iw, coeff: float, stream) -> None:
    """The (user, positive) reg-gradient rows: n copies of kreg * W[r] per row with n keys."""
    _ffi.check(lib.lgcn_reg_rows_add(st.fixed_sparse.rowptr.data_ptr(), st.reg_rows.data_ptr(), st.reg_rows.numel(),
                                     uw.data_ptr(), iw.data_ptr(), U, d, coeff, st.B, gu.data_ptr(), gi.data_ptr(), U,
                                     stream), "lgcn_reg_rows_add")


class FusedTrainStep:
    """Callable training step for a LightGCN model (models.light_gcn.LightGCN).

    step(batch) -> device loss tensor [1]: gradients, optional DP all-reduce, optimizer step.
    compute_grads(batch) -> loss: sets user/item_embedding.weight.grad only."""

    def __init__(self, model, optimizer, bpr_coeff: float = 5e-3, world: int = 1, max_entries: int = 1024,
                 graphs: bool = False, lazy: bool = False, exchange=None, neg_seed: int | None = None,
                 cols: ColumnGroup | None = None, neg_sampler=None, loss_acc: torch.Tensor | None = None):
        """graphs=True: the first step of each batch runs eagerly, then the whole step (gradients
        and, at world == 1, the optimizer — which must be a capturable FusedAdam) is captured in a
        per-batch hipGraph and replayed from then on; negatives still come from the global CUDA
        generator (graph-safe Philox offsets), so each replay draws new ones.
        exchange (lazy, data parallel): a lgcn_amd.distributed.RowExchange (replicated optimizer;
        the step is two captured halves around the eager all_gather of the packed gradient rows), a
        lgcn_amd.distributed.HybridExchange (the same, the item gradient table all_reduced whole:
        large batches) or a lgcn_amd.owner.OwnerExchange (owner-sharded optimizer:
        step(batch, next_batch) — the rows of next_batch's step are fetched from their owners at
        the end of this one).
        neg_seed: draw step k's negatives from a generator seeded (neg_seed, k) instead of the
        global CUDA generator (the same draws whichever exchange runs, and whenever they are drawn).
        cols (lazy): column-sharded training — the model holds this rank's ColumnGroup columns,
        every rank steps the same batches with the same negatives (the same neg_seed); with graphs,
        each batch's step is captured as graphs cut at the two collectives (_SegmentedGraph).
        neg_sampler (pos_items [B] -> item ids [B]): draw the negatives with it (the harness passes
        utils.helpers.sample_negative, so what that function draws — patched or not — is what the
        step trains on); default: torch.randint(0, I, (B,)) into the batch's buffer, the same draws.
        loss_acc (lazy; device float64 [1]): each step adds double(loss) * its batch's edge count to
        it (lgcn_loss_accumulate, inside the captured step) — the harness's epoch-loss sum."""
        self.model = model
        self.optimizer = optimizer
        self.coeff = float(bpr_coeff)
        self.world = world
        self.max_entries = max_entries
        self.graphs = graphs
        self.lazy = lazy
        self.exchange = exchange
        if lazy:
            from .optim import RowLazyAdam

            if not isinstance(optimizer, RowLazyAdam):
                raise ValueError("lazy=True needs a lgcn_amd.optim.RowLazyAdam")
            if world > 1 and exchange is None:
                raise ValueError("lazy=True with world > 1 needs a lgcn_amd.distributed.RowExchange")
        elif graphs and world == 1 and not getattr(optimizer, "capturable", False):
            raise ValueError("graphs=True needs a capturable optimizer (lgcn_amd.optim.FusedAdam(capturable=True))")
        # per-batch states (plans, buffers, captured graphs) by batch content: a loader that
        # collates a new edge_index each epoch (the reference's PyG DataLoader) still replays
        from ._cache import ContentLRU

        self._states = ContentLRU(max_entries)
        from .owner import OwnerExchange

        self.cols = cols
        if cols is not None:
            if not lazy or exchange is not None:
                raise ValueError("cols= needs lazy=True (RowLazyAdam) and no exchange")
            if model.dim_h != cols.d:
                raise ValueError(f"the model holds {model.dim_h} columns, the ColumnGroup share is {cols.d}")
        self.owner = isinstance(exchange, OwnerExchange)
        self.hybrid = getattr(exchange, "dense_items", False)
        if self.owner and not lazy:
            raise ValueError("an OwnerExchange needs lazy=True (RowLazyAdam)")
        self.neg_seed = neg_seed
        self.neg_sampler = neg_sampler
        if loss_acc is not None and (loss_acc.dtype != torch.float64 or loss_acc.numel() < 1 or not lazy):
            raise ValueError("loss_acc must be a device float64 tensor of >= 1 element (lazy=True)")
        self.loss_acc = loss_acc
        # one GPU, whole rows: the BPR reg-gradient rows go into the clip norm and the update
        # (lgcn_row_*_reg) instead of two passes after the backward — bitwise the same step
        from . import tuning

        self.reg_in_update = bool(lazy and exchange is None and cols is None and tuning.get().reg_in_update)
        self._gen = None
        self._k = 0  # steps taken (the index of the next step)
        self._owner_graphs = None
        self._synced = True  # every row current on every rank (start, or after sync())

    def state(self, edge_index: torch.Tensor) -> _BatchState:
        """The batch's state, built on the first step of a batch of this content (lgcn_amd._cache:
        the same tensor object without hashing, else by content; least recently used evicted
        beyond max_entries)."""
        return self._states.get(edge_index, lambda: _BatchState(self.model, edge_index, self.model.dim_h,
                                                                 lazy=self.lazy))

    def drop_graphs(self) -> None:
        """Forget every batch's captured hipGraph (the next step of each batch recaptures it):
        needed when a buffer a graph reads moved, e.g. RowLazyAdam.reserve() grew its constants."""
        for st in self._states.values():
            for a in ("graph", "graph_post", "graph_loss", "graph_grads"):
                if hasattr(st, a):
                    setattr(st, a, None)
        self._owner_graphs = None  # the owner update's graph reads the optimizer's constants too

    def has_state(self, edge_index: torch.Tensor) -> bool:
        """A state for a batch of this content exists (its checks already passed)."""
        return self._states.key_of(edge_index) in self._states

    def _draw(self, st, k: int | None = None) -> None:
        """Step k's negatives (reference utils/helpers.py:64-82: torch.randint(0, I, (B,))).
        Graph replays draw them eagerly just before the replay: a captured draw makes every
        replay launch the generator's seed/offset fills first (two small kernels, ~9 us per C3
        step, profiles/r02zz_graph_rng/), and the values are the same draws either way."""
        m = self.model
        dev = m.user_embedding.weight.device
        k = self._k if k is None else k
        if self.neg_sampler is not None:
            if hasattr(self.neg_sampler, "draw_into"):
                self.neg_sampler.draw_into(st.neg, st.pos)
            else:
                st.neg.copy_(self.neg_sampler(st.pos))
            st.neg_step = k
            return
        gen = None
        if self.neg_seed is not None:
            if self._gen is None:
                self._gen = torch.Generator(device=dev)
            self._gen.manual_seed(int(self.neg_seed) * 1_000_003 + int(k))
            gen = self._gen
        torch.randint(0, m.num_items, (st.B,), device=dev, out=st.neg, generator=gen)
        st.neg_step = k

    def compute_grads(self, batch, draw: bool = True) -> torch.Tensor:
        m = self.model
        ei = batch.edge_index
        st = self.state(ei)
        lib = _ffi.load()
        uw, iw = m.user_embedding.weight, m.item_embedding.weight
        U, I, K, d = m.num_users, m.num_items, m.num_layers, m.dim_h
        N = U + I
        B = st.B
        dev = uw.device
        stream = _ffi.stream_of(dev)
        div = float(K + 1)
        mul = float(np.float32(1.0 / (K + 1)))
        with torch.no_grad():
            if draw:
                self._draw(st)
            out = propagate_forward(uw.detach(), iw.detach(), st.plan, K)
            if not st.small:  # only the all-keys sort reads the negatives' global row keys
                torch.add(st.neg, U, out=st.keys[2 * B:])
            _ffi.check(lib.lgcn_bpr_fused(out.data_ptr(), None, N, uw.data_ptr(), iw.data_ptr(), U, U,
                                          st.users.data_ptr(), st.pos.data_ptr(), st.neg.data_ptr(), B, d,
                                          st.plan.touched.data_ptr(), div, mul,
                                          self.coeff, st.cf.data_ptr(), _ffi.ptr(st.cw), st.terms.data_ptr(),
                                          stream), "lgcn_bpr_fused")
            fused = st.small and loss_fused(st, I)
            if not fused:
                _ffi.check(lib.lgcn_bpr_loss(st.terms.data_ptr(), B, d, self.coeff, st.loss.data_ptr(),
                                             st.loss_part.data_ptr(), stream),
                           "lgcn_bpr_loss")
            gu = torch.empty((U, d), dtype=torch.float32, device=dev)
            gi = torch.empty((I, d), dtype=torch.float32, device=dev)
            grads = (gu, gi, U)
            if st.small:
                # g = (dF * mul) / div: fixed rows through the per-batch plan (every row written, 0 if
                # empty), then the negatives' rows sorted in one workgroup and added run by run
                big = 1 << 62
                spmm(st.fixed_dense, N, d, (st.cf, None, big), None, grads, None, _ffi.EPI_SCALE, div, mul,
                     stream=stream)
                # negatives: dF rows into g now, their reg rows parked (per row, first-occurrence slot)
                scatter_negatives(lib, st, gu, gi, U, I, d, mul, div, None, stream, uw, iw, self.coeff,
                                  (st.terms, d, self.coeff, st.loss) if fused else None)
                propagate_backward_seeded(gu, gi, st.plan, K)
                add_fixed_reg_rows(lib, st, gu, gi, U, N, d, uw, iw, self.coeff, stream)
                add_negative_reg_rows(lib, st, gu, gi, U, d, uw, iw, self.coeff, stream)
            else:
                # large batches: one stable radix sort of all 3B row keys per step
                _ffi.check(lib.lgcn_csr_build(st.keys.data_ptr(), st.keys.data_ptr(), 3 * B, N, st.rowptr.data_ptr(),
                                              st.col.data_ptr(), st.eid.data_ptr(), st.err.data_ptr(),
                                              st.ws.data_ptr(), st.ws.numel(), stream), "lgcn_csr_build")
                _ffi.check(lib.lgcn_segment_rows(st.rowptr.data_ptr(), st.eid.data_ptr(), st.cf.data_ptr(), N, d,
                                                 gu.data_ptr(), gi.data_ptr(), U, 0, mul, div, stream),
                           "lgcn_segment_rows")
                propagate_backward_seeded(gu, gi, st.plan, K)
                _ffi.check(lib.lgcn_segment_rows(st.rowptr.data_ptr(), st.eid.data_ptr(), st.cw.data_ptr(), N, d,
                                                 gu.data_ptr(), gi.data_ptr(), U, 1, 1.0, 1.0, stream),
                           "lgcn_segment_rows")
        uw.grad = gu
        iw.grad = gi
        return st.loss

    def _bpr(self, lib, st, out, uw, iw, U: int, N: int, B: int, d: int, div: float, mul: float, stream) -> float:
        """The fused cosine-BPR kernel and the loss sum; returns the reg coefficient the scatters'
        reg rows use. Column-sharded: this rank's partial sums, one all_reduce of [B, 6] over the
        column groups, then the gradient rows of its columns from the full sums."""
        c = self.cols
        if c is None:
            _ffi.check(lib.lgcn_bpr_fused(out.data_ptr(), None, N, uw.data_ptr(), iw.data_ptr(), U, U,
                                          st.users.data_ptr(), st.pos.data_ptr(), st.neg.data_ptr(), B, d,
                                          st.plan.touched.data_ptr(), div, mul,
                                          self.coeff, st.cf.data_ptr(), _ffi.ptr(st.cw), st.terms.data_ptr(),
                                          stream), "lgcn_bpr_fused")
            if not loss_fused(st, N - U):  # else the range scatter's launch sums it (_step_lazy)
                _ffi.check(lib.lgcn_bpr_loss(st.terms.data_ptr(), B, d, self.coeff, st.loss.data_ptr(),
                                             st.loss_part.data_ptr(), stream), "lgcn_bpr_loss")
            return self.coeff
        if getattr(st, "sums", None) is None:
            st.sums = torch.empty(max(1, 6 * B), dtype=torch.float32, device=uw.device)
        args = (out.data_ptr(), None, N, uw.data_ptr(), iw.data_ptr(), U, U, st.users.data_ptr(), st.pos.data_ptr(),
                st.neg.data_ptr(), B, d, c.d_full, st.plan.touched.data_ptr(), div, mul, self.coeff,
                st.sums.data_ptr())
        _ffi.check(lib.lgcn_bpr_fused_cols(*args, 1, None, None, None, stream), "lgcn_bpr_fused_cols(partials)")
        c.all_reduce(st.sums)
        _ffi.check(lib.lgcn_bpr_fused_cols(*args, 2, st.cf.data_ptr(), _ffi.ptr(st.cw), st.terms.data_ptr(), stream),
                   "lgcn_bpr_fused_cols")
        _ffi.check(lib.lgcn_bpr_loss(st.terms.data_ptr(), B, c.d_full, self.coeff, st.loss.data_ptr(),
                                     st.loss_part.data_ptr(), stream), "lgcn_bpr_loss")
        return c.reg_coeff(self.coeff)

    def _step_lazy(self, st: _BatchState, draw: bool = True) -> torch.Tensor:
        """The whole batch step with the row-lazy optimizer: catch the batch's rows (touched rows
        and this step's negatives) up, forward, loss, gradient rows written only where the step
        can make them nonzero, backward, [row exchange], clip + Adam on exactly those rows."""
        loss = self._lazy_grads(st, draw)
        if self.exchange is not None:
            self.exchange.gather()
        self._lazy_update(st)
        return loss

    def _lazy_grads(self, st: _BatchState, draw: bool = True) -> torch.Tensor:
        m = self.model
        opt = self.optimizer
        lib = _ffi.load()
        uw, iw = m.user_embedding.weight, m.item_embedding.weight
        U, I, K, d = m.num_users, m.num_items, m.num_layers, m.dim_h
        N = U + I
        B = st.B
        dev = uw.device
        stream = _ffi.stream_of(dev)
        div = float(K + 1)
        mul = float(np.float32(1.0 / (K + 1)))
        big = 1 << 62
        with torch.no_grad():
            if draw:
                self._draw(st)
            if not self.owner:  # owner-sharded: the rows were fetched current by the previous step
                opt.catch_up(st.touched_rows, st.neg, U)
            out = propagate_forward(uw.detach(), iw.detach(), st.plan, K)
            reg_coeff = self._bpr(lib, st, out, uw, iw, U, N, B, d, div, mul, stream)
            gu, gi = opt.gu, opt.gi
            if self.hybrid:  # the whole item table is all_reduced: rows this step leaves alone are 0
                gi.zero_()
            grads = (gu, gi, U)
            # seed g = (dF * mul) / div on every touched row (0 where no (user, positive) key)...
            spmm(st.fixed_touched, N, d, (st.cf, None, big), None, grads, None, _ffi.EPI_SCALE, div, mul,
                 stream=stream)
            # ... the negatives' rows added (stored where the row is outside the touched set)
            fused = loss_fused(st, I, self.cols)
            # the harness's epoch-loss sum rides in the same workgroup as the fused loss (counted
            # range scatter), else lgcn_loss_accumulate at the end of the step
            acc_fused = self.loss_acc is not None and fused and self.reg_in_update
            scatter_negatives(lib, st, gu, gi, U, I, d, mul, div, st.plan.touched, stream, uw, iw, reg_coeff,
                              (st.terms, d, self.coeff, st.loss) if fused else None, counts=self.reg_in_update,
                              loss_acc=(self.loss_acc, float(st.n_edges)) if acc_fused else None)
            propagate_backward_seeded(gu, gi, st.plan, K)
            if not self.reg_in_update:  # else _lazy_update's norm and update form them (_reg_rows)
                add_fixed_reg_rows(lib, st, gu, gi, U, N, d, uw, iw, reg_coeff, stream)
                add_negative_reg_rows(lib, st, gu, gi, U, d, uw, iw, reg_coeff, stream)
            ex = self.exchange
            if self.owner:
                # this rank's rows with a possibly nonzero gradient -> their owners' blocks
                _ffi.check(lib.lgcn_owner_reset(ex.send.data_ptr(), ex.world, ex.blk, ex.cap, ex.req_off, ex.rcap,
                                                ex.counts.data_ptr(), stream), "lgcn_owner_reset")
                _ffi.check(lib.lgcn_owner_pack_rows(gu.data_ptr(), gi.data_ptr(), U, d, st.touched_rows.data_ptr(),
                                                    st.touched_rows.numel(), st.neg.data_ptr(), B, U,
                                                    st.c2flag.data_ptr(), st.plan.touched.data_ptr(), ex.world,
                                                    ex.cap, ex.blk, ex.counts.data_ptr(), ex.send.data_ptr(),
                                                    ex.overflow.data_ptr(), stream), "lgcn_owner_pack_rows")
            elif self.hybrid:
                # the users' rows -> the record slots (the item table goes whole, all_reduced)
                _ffi.check(lib.lgcn_rows_pack(gu.data_ptr(), gi.data_ptr(), U, d, st.touched_users.data_ptr(),
                                              st.touched_users.numel(), None, 0, U, None, None, ex.cap,
                                              ex.ids.data_ptr(), ex.rows.data_ptr(), stream), "lgcn_rows_pack(users)")
            elif ex is not None:
                # this rank's rows with a possibly nonzero gradient -> the exchange slots
                _ffi.check(lib.lgcn_rows_pack(gu.data_ptr(), gi.data_ptr(), U, d, st.touched_rows.data_ptr(),
                                              st.touched_rows.numel(), st.neg.data_ptr(), B, U,
                                              st.c2flag.data_ptr(), st.plan.touched.data_ptr(), ex.cap,
                                              ex.ids.data_ptr(), ex.rows.data_ptr(), stream), "lgcn_rows_pack")
            if self.loss_acc is not None and not acc_fused:
                _ffi.check(lib.lgcn_loss_accumulate(st.loss.data_ptr(), float(st.n_edges), self.loss_acc.data_ptr(),
                                                    stream), "lgcn_loss_accumulate")
        return st.loss

    def _reg_rows(self, st: _BatchState):
        """The step's BPR reg-gradient rows by occurrence counts (lgcn_reg_rows_t): the fixed
        (user, positive) counts from the batch's segment plan, the negatives' from the sorted path's
        grouping or the range scatter's st.neg_count; kreg = coeff * 2 / (B * d) from the tables."""
        if st.B == 0:
            return None
        m = self.model
        U = m.num_users
        return _ffi.RegRows(w_lo=m.user_embedding.weight.data_ptr(), w_hi=m.item_embedding.weight.data_ptr(),
                            w_split=U, coeff=self.coeff, B=st.B, fixed_rowptr=st.fixed_sparse.rowptr.data_ptr(),
                            neg_rowptr=_ffi.ptr(st.neg_rowptr),
                            neg_count=None if st.neg_rowptr is not None else st.neg_count.data_ptr(),
                            neg_off=U, neg_rows=m.num_items)

    def _lazy_update(self, st: _BatchState) -> None:
        """Clip + Adam on the rows whose gradient can be nonzero: this rank's (touched rows, then
        negatives at their first occurrence that are not touched), or with an exchange the union
        of every rank's, summed in rank order and divided by W."""
        opt = self.optimizer
        ex = self.exchange
        with torch.no_grad():
            if ex is None:
                opt.step_rows(st.touched_rows, st.neg, self.model.num_users, first_b=st.c2flag,
                              skip_b=st.plan.touched,
                              gather_partials=self.cols.gather_partials if self.cols is not None else None,
                              reg=self._reg_rows(st) if self.reg_in_update else None)
                return
            lib = _ffi.load()
            m = self.model
            stream = _ffi.stream_of(ex.ids_all.device)
            n = ex.world * ex.cap
            ex.unpack_ids()
            _ffi.check(lib.lgcn_rows_mark_first(ex.ids_all.data_ptr(), n, ex.claim.data_ptr(), ex.first.data_ptr(),
                                                stream), "lgcn_rows_mark_first")
            _ffi.check(lib.lgcn_rows_accumulate(ex.ids_all.data_ptr(), ex.rows_ptr(), ex.world, ex.cap, ex.blk,
                                                ex.first.data_ptr(), opt.gu.data_ptr(), opt.gi.data_ptr(),
                                                m.num_users, m.dim_h, float(ex.world), stream),
                       "lgcn_rows_accumulate")
            if self.hybrid:
                # the all_reduced item sums / W (as lgcn_rows_accumulate divides), then every item row
                # and the union of the users' rows
                opt.gi.div_(float(ex.world))
                opt.step_rows(ex.items_all, ex.ids_all, 0, first_b=ex.first)
                return
            opt.step_rows(None, ex.ids_all, 0, first_b=ex.first)

    # --- owner-sharded exchange (lgcn_amd.owner) ----------------------------------------------
    def _owner_reduce(self) -> None:
        """Owner side, after the blocks arrived: the received gradient rows summed per row in rank
        order / W, and this rank's clip-norm partials over its rows of the union (row order)."""
        ex, opt, m = self.exchange, self.optimizer, self.model
        lib = _ffi.load()
        stream = _ffi.stream_of(ex.ids_all.device)
        ex.unpack()
        n = ex.world * ex.cap
        _ffi.check(lib.lgcn_rows_mark_first(ex.ids_all.data_ptr(), n, ex.claim.data_ptr(), ex.first.data_ptr(),
                                            stream), "lgcn_rows_mark_first")
        _ffi.check(lib.lgcn_rows_accumulate(ex.ids_all.data_ptr(), ex.rows_ptr(), ex.world, ex.cap, ex.blk,
                                            ex.first.data_ptr(), opt.gu.data_ptr(), opt.gi.data_ptr(), m.num_users,
                                            m.dim_h, float(ex.world), stream), "lgcn_rows_accumulate")
        if opt.max_grad_norm is not None:
            _ffi.check(lib.lgcn_rows_mark(ex.ids_all.data_ptr(), ex.first.data_ptr(), n, ex.not_union.data_ptr(), 0,
                                          stream), "lgcn_rows_mark")
            opt.sqnorm_partials(ex.owned, ex.not_union, ex.partials)
            _ffi.check(lib.lgcn_rows_mark(ex.ids_all.data_ptr(), ex.first.data_ptr(), n, ex.not_union.data_ptr(), 1,
                                          stream), "lgcn_rows_mark")

    def _owner_update(self) -> None:
        """Owner side: the Adam step on its rows of the union, then the requested rows caught up
        to the new step and copied into the reply blocks."""
        ex, opt, m = self.exchange, self.optimizer, self.model
        lib = _ffi.load()
        stream = _ffi.stream_of(ex.ids_all.device)
        opt.step_rows_with_partials(ex.ids_all, ex.first,
                                    ex.partials_all if opt.max_grad_norm is not None else None)
        opt.catch_up(None, ex.req_all, 0, first_b=ex.req_valid)
        _ffi.check(lib.lgcn_rows_gather(opt.uw.data_ptr(), opt.iw.data_ptr(), m.num_users, m.dim_h,
                                        ex.req_all.data_ptr(), ex.req_all.numel(), ex.reply_send.data_ptr(), 0,
                                        stream), "lgcn_rows_gather(replies)")

    def _step_owner(self, st: _BatchState, nxt: _BatchState | None) -> torch.Tensor:
        ex, opt, m = self.exchange, self.optimizer, self.model
        lib = _ffi.load()
        U = m.num_users
        stream = _ffi.stream_of(m.user_embedding.weight.device)
        if ex.pending is not st and not self._synced:
            raise RuntimeError("OwnerExchange: this batch's rows were not fetched by the previous step (pass "
                               "next_batch to step(), or call sync() before a step out of order)")
        if getattr(st, "neg_step", None) != self._k:
            self._draw(st, self._k)
        use_graphs = self.graphs
        if use_graphs and getattr(st, "graph", None) is not None:
            st.graph.replay()
            loss = st.graph_loss
        else:
            loss = self._lazy_grads(st, draw=False)
            if use_graphs:
                torch.cuda.synchronize()
                program = _programs_on()
                g = _new_graph(program)
                with torch.cuda.graph(g):
                    st.graph_loss = self._lazy_grads(st, draw=False)
                st.graph = _replayable(g, program)
        # the next step's rows: its batch's touched rows and its negatives, drawn now
        ex.mine.fill_(-1)
        if nxt is not None:
            self._draw(nxt, self._k + 1)
            ex.req_stamp = (ex.req_stamp + 1) % (2**31 - 1)
            if ex.req_stamp == 0:  # wrapped: no stale stamp may equal a new one
                ex.req_claim.fill_(-1)
                ex.req_stamp = 1
            _ffi.check(lib.lgcn_owner_pack_requests(nxt.touched_rows.data_ptr(), nxt.touched_rows.numel(),
                                                    nxt.neg.data_ptr(), nxt.B, U, ex.world, ex.rcap, ex.blk,
                                                    ex.req_off, ex.counts.data_ptr(), ex.send.data_ptr(),
                                                    ex.mine.data_ptr(), ex.overflow.data_ptr(),
                                                    ex.req_claim.data_ptr(), ex.req_stamp, stream),
                       "lgcn_owner_pack_requests")
        ex.exchange_blocks()
        graphs_ok = use_graphs and self._owner_graphs is not None
        if graphs_ok:
            self._owner_graphs[0].replay()
        else:
            self._owner_reduce()
        if opt.max_grad_norm is not None:
            ex.gather_partials()
        if graphs_ok:
            if opt.steps + 1 > opt.max_steps:
                raise RuntimeError(f"RowLazyAdam: more than max_steps={opt.max_steps} steps")
            self._owner_graphs[1].replay()
            opt.steps += 1
        else:
            self._owner_update()
        ex.exchange_replies()
        _ffi.check(lib.lgcn_rows_gather(opt.uw.data_ptr(), opt.iw.data_ptr(), U, m.dim_h, ex.mine.data_ptr(),
                                        ex.mine.numel(), ex.reply_recv.data_ptr(), 1, stream),
                   "lgcn_rows_gather(scatter replies)")
        if use_graphs and self._owner_graphs is None:
            # the owner's two halves touch only the exchange buffers: one capture serves every batch
            torch.cuda.synchronize()
            steps = opt.steps
            program = _programs_on()
            g0, g1 = _new_graph(program), _new_graph(program)
            # the capture records the launches of the step just run and runs none: its max_steps
            # check is taken at that step's index (not one past it, which fails when the table is
            # exactly full), and the count is restored after
            opt.steps = steps - 1
            try:
                with torch.cuda.graph(g0):
                    self._owner_reduce()
                with torch.cuda.graph(g1):
                    self._owner_update()
            finally:
                opt.steps = steps
            self._owner_graphs = (_replayable(g0, program), _replayable(g1, program))
        ex.pending = nxt
        self._synced = False
        self._k += 1
        if not getattr(st, "owner_checked", False):
            # the blocks are sized so that neither list overflows (owner_capacity); the first step
            # of each batch state checks that with one host read, so a dropped row is an error at
            # once rather than at the next check_overflow()
            ex.check_overflow()
            st.owner_checked = True
        return loss

    def sync(self) -> None:
        """Make the parameters current (row-lazy optimizer: replay every deferred row; owner-sharded:
        every owner replays its rows, then one all_gather of the owned rows)."""
        if self.owner:
            ex, opt, m = self.exchange, self.optimizer, self.model
            opt.catch_up(None, ex.owned, 0)
            ex.all_gather_owned(opt.uw, opt.iw, m.num_users)
            self._synced = True
            return
        if self.lazy:
            self.optimizer.flush()

    def check_overflow(self) -> None:
        """Raise if any step's negative scatter overflowed a workgroup list, or (owner-sharded) a
        destination block (never expected for uniform negatives; one host read per batch state —
        call once per epoch)."""
        if self.owner:
            self.exchange.check_overflow()
        for st in self._states.values():
            if getattr(st, "overflow", None) is not None and int(st.overflow.item()):
                raise RuntimeError("lgcn_range_scatter_add overflowed: negatives too concentrated for its lists")
            if getattr(st, "neg_err", None) is not None and int(st.neg_err.item()):
                # the grouping's integrity checks (lgcn_group_keys: >= 2^32) or an out-of-range key
                raise RuntimeError(f"negatives grouping reported errors ({int(st.neg_err.item()):#x})")

    def _optimize(self) -> None:
        if getattr(self.optimizer, "fused_clip_norm", None) is None:
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), max_norm=1)
        self.optimizer.step()

    def _allreduce(self) -> None:
        from .distributed import allreduce_grads

        allreduce_grads([self.model.user_embedding.weight, self.model.item_embedding.weight], self.world)

    def step(self, batch, next_batch=None) -> torch.Tensor:
        """One training step on batch. next_batch (owner-sharded: the batch the NEXT step will
        take): its rows are fetched from their owners at the end of this step."""
        if self.owner:
            st = self.state(batch.edge_index)
            nxt = self.state(next_batch.edge_index) if next_batch is not None else None
            if not st.lazy or (nxt is not None and not nxt.lazy):
                raise ValueError("lazy step needs a batch whose 3B contribution ids fit int32 (3B < 2^31)")
            return self._step_owner(st, nxt)
        loss = self._step_replicated(batch)
        self._k += 1
        return loss

    def _step_replicated(self, batch) -> torch.Tensor:
        if self.lazy:
            st = self.state(batch.edge_index)
            if not st.lazy:
                raise ValueError("lazy step needs a batch whose 3B contribution ids fit int32 (3B < 2^31)")
            if not self.graphs:
                return self._step_lazy(st)
            if getattr(st, "graph", None) is None:
                loss = self._step_lazy(st)  # real first step (warms allocations), then capture
                torch.cuda.synchronize()
                steps = self.optimizer.steps
                # issued as launch programs (StepProgram) unless tuned off
                program = _programs_on()
                g = _new_graph(program)
                # the capture records the launches of the step just run and runs none: its
                # max_steps check is taken at that step's index (one past it fails when the
                # constant table is exactly full), and the count is restored after
                self.optimizer.steps = steps - 1
                try:
                    if self.cols is not None and self.cols.world > 1:
                        # graphs cut at the column groups' two collectives, which run eagerly between them
                        g = _SegmentedGraph()
                        self.cols.capture = g
                        try:
                            st.graph_loss = g.capture(lambda: self._step_lazy(st, draw=False))
                        finally:
                            self.cols.capture = None
                    elif self.exchange is None:
                        with torch.cuda.graph(g):
                            st.graph_loss = self._step_lazy(st, draw=False)
                    else:  # two halves: the all_gather between them runs eagerly
                        with torch.cuda.graph(g):
                            st.graph_loss = self._lazy_grads(st, draw=False)
                        post = _new_graph(program)
                        with torch.cuda.graph(post):
                            self._lazy_update(st)
                        st.graph_post = _replayable(post, program)
                finally:
                    self.optimizer.steps = steps
                st.graph = g if isinstance(g, _SegmentedGraph) else _replayable(g, program)
                return loss
            if self.optimizer.steps + 1 > self.optimizer.max_steps:
                raise RuntimeError("RowLazyAdam: max_steps exceeded")
            self._draw(st)
            st.graph.replay()
            if self.exchange is not None:
                self.exchange.gather()
                st.graph_post.replay()
            self.optimizer.steps += 1
            return st.graph_loss
        if not self.graphs:
            loss = self.compute_grads(batch)
            if self.world > 1:
                self._allreduce()
            self._optimize()
            return loss
        st = self.state(batch.edge_index)
        if getattr(st, "graph", None) is None:
            # real first step (warms every allocation and the optimizer state), then capture
            loss = self.compute_grads(batch)
            if self.world > 1:
                self._allreduce()
            self._optimize()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                st.graph_loss = self.compute_grads(batch, draw=False)
                st.graph_grads = (self.model.user_embedding.weight.grad, self.model.item_embedding.weight.grad)
                if self.world == 1:
                    self._optimize()
            st.graph = g
            return loss
        self._draw(st)
        st.graph.replay()
        m = self.model
        m.user_embedding.weight.grad, m.item_embedding.weight.grad = st.graph_grads
        if self.world > 1:
            self._allreduce()
            self._optimize()
        return st.graph_loss
