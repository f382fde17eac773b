"""Propagation plans: the device-resident CSR + gcn_norm weights + load-balanced schedule that
one ``edge_index`` needs, built once and reused by every layer and every step.

The reference re-derives all of this inside every LGConv call (PyG 2.4.0 ``gcn_norm`` +
``propagate``, reached from reference models/light_gcn.py:33), K times per forward; the
result is identical each time, so a plan per edge set is a legal cache.

HBM layout of one direction (``CsrDirection``), E edges, N nodes:
    rowptr int64[N+1] | col int32[E] | val fp32[E] | eid int32[E] (edge position, tests/debug)
    items  lgcn_item_t[cap] (16 B)    | splits lgcn_split_t[N] (16 B)
The forward direction has rows = targets (edge_index[1]); the transposed direction (built
lazily, only when autograd needs it) has rows = sources (edge_index[0]). Both keep the input
edge order inside a row, which is the order CPU scatter_add_/index_add_ add in.
"""
from __future__ import annotations

import dataclasses

import torch

from . import _ffi

DEFAULT_CHUNK = 256
# hub chunk of the source-sliced schedule: a chunk is one lane group's sequential chain (one L2
# latency per 8 edges), and every slice launch waits for its longest chain, while shorter chunks
# make more partials. Re-swept after the index rounds and non-temporal rows (profiles/r02zg/,
# interleaved): C2 K=3 d=64 1.238 ms at 128, 1.225 at 160, 1.217 at 192, 1.235 at 224, 1.240 at
# 256; d=32 within 1 % from 128 to 256.
SLICED_CHUNK = 192
# hub chunk of the plain schedule the sharded forward's ranks run when R > 1 (lgcn_amd.sharded.
# rank_chunk): per-rank K=3 step at 8 x 1 0.246 ms at 128, 0.253 at 256 (profiles/r02k_shard/)
RANK_CHUNK = 128


def sliced_chunk(chunk: int) -> int:
    return min(int(chunk), SLICED_CHUNK)
# batch plans (touched-only, segment) use the one-launch block-split schedule (C3 step 0.222 ->
# 0.203 ms, profiles/r01l_blocksplit/) ...
# ... while no split row has more chunks than this: lgcn_spmm_blocksplit sums a split row in one
# workgroup (16 running sums, csrc/lgcn_spmm.hip kVSums), so a row of c chunks is a chain of
# ceil(c / 16) chunks — the launch's critical path. Past 2 chunks per running sum (a structured
# graph's big batches: hub rows with thousands of intra-batch edges) the item pass + combine pair
# (every chunk in parallel, the same association, so the same bits) is faster.
BLOCK_SPLIT_MAX_CHUNKS = 32


def _block_split_for(splits: torch.Tensor, n_splits: int) -> bool:
    return n_splits == 0 or int(splits[:n_splits, 2].max().item()) <= BLOCK_SPLIT_MAX_CHUNKS


def slice_bytes_for(num_nodes: int, d: int) -> int:
    """Source-slice size for a full-graph propagation of width d (0 = no slicing). Measured on
    the C2 graph (tools/sliced_probe.py, profiles/r01g_sliced): slicing pays while the gathered
    table is small enough that re-reading the running row sums once per slice costs less than the
    cache misses it saves — about 8 slices of 8–24 MB for tables of 16–512 MB, 2-3 slices of 4-12
    MB for the 4-32 MB tables of the narrow column shares (d = 8-32); beyond 512 MB (C5: 11 GB)
    the plain schedule is faster. PropagationPlan.schedule also requires >= 8 edges per
    row per slice. lgcn_amd.tuning's slice_mb overrides the size and that density test (0
    disables)."""
    from . import tuning

    v = tuning.get().slice_mb
    if v is not None:
        return int(v * 2**20) if v > 0 else 0
    x = int(num_nodes) * int(d) * 4
    if x < 4 * 2**20 or x > 512 * 2**20:
        return 0
    if x < 8 * 2**20:
        # 4-8 MB tables (C2 at d = 8, the 1 x 8 grid's column share): 4 MB slices (bench.py --dim 8:
        # 0.775 plain -> 0.721 ms; 3 MB 0.727, 6 MB 0.731, profiles/r05zd_narrow/)
        return 4 * 2**20
    if x < 16 * 2**20:
        # 8-16 MB tables (C2 at d = 16, the 1 x 4 grid's column share): 8 MB slices, 2 user + 1
        # item (bench.py --dim 16: 0.6175 plain -> 0.6026 ms per K=3 step; 6 MB 0.6020, 12 MB
        # 0.6122, profiles/r05zd_narrow/)
        return 8 * 2**20
    if x < 32 * 2**20:
        # 16-32 MB tables (C2 at d = 32, the 1 x 2 grid's column share): 12 MB slices, i.e. 2 user +
        # 1 item slice, beat 8 MB's 3 + 1 (bench.py --dim 32: 0.710 -> 0.690 ms per K=3 step,
        # profiles/r02zz_narrow/; round 5: 0.667 at 12 MB vs 0.686 / 0.671 / 0.751 / 0.791 at 8 /
        # 16 / 24 MB / plain, profiles/r05zd_narrow/)
        return 12 * 2**20
    return int(min(max(x // 8, 8 * 2**20), 24 * 2**20))


@dataclasses.dataclass
class CsrDirection:
    rowptr: torch.Tensor
    col: torch.Tensor
    eid: torch.Tensor
    val: torch.Tensor
    items: torch.Tensor   # int64 [cap, 2] viewed as lgcn_item_t
    splits: torch.Tensor  # int32 [N, 4] viewed as lgcn_split_t
    n_items: int
    n_splits: int
    n_partials: int
    chunk: int
    # one-launch schedule (lgcn_spmm_blocksplit): split rows summed by one workgroup each, in the
    # combine pass's association. For plans whose split rows have few chunks (batch plans).
    block_split: bool = False

    def block_lists(self):
        """(row items [n, 2] int64, n, chunk items [n_partials, 2] in partial-slot order) for
        lgcn_spmm_blocksplit; built on first use (one host sync) and cached."""
        cached = getattr(self, "_block_lists", None)
        if cached is None:
            it = self.items[: self.n_items]
            dst = it[:, 1].contiguous().view(torch.int32).view(-1, 2)[:, 1]
            part = dst < 0
            rows = it[~part].contiguous()
            chunks = torch.empty((max(self.n_partials, 1), 2), dtype=torch.int64, device=it.device)
            chunks[(-dst[part] - 1).long()] = it[part]
            cached = self._block_lists = (rows, int(rows.shape[0]), chunks)
        return cached

    def item_table(self) -> torch.Tensor:
        """Items as int64 [n_items, 3] = (beg, len, dst) — for tests."""
        it = self.items[: self.n_items]
        lens_dst = it[:, 1].contiguous().view(torch.int32).view(-1, 2)
        return torch.stack([it[:, 0], lens_dst[:, 0].long(), lens_dst[:, 1].long()], dim=1)


SMALL_SPLIT_CHUNKS = 16  # kVSums (csrc/lgcn_spmm.hip): a split row of <= this many chunks combines in a lane group


def pack_split_rows(direction: CsrDirection) -> int:
    """Order the direction's split rows big-first (more than SMALL_SPLIT_CHUNKS chunks) and record
    how many are big (direction.n_split_big, lgcn_pass_t.n_split_big): the pair combine then gives
    each big row a workgroup and packs the small ones one per lane group. The combine reads a row's
    partials through its split record, so the order changes nothing else (one host sync)."""
    n = direction.n_splits
    if n == 0:
        direction.n_split_big = 0
        return 0
    sp = direction.splits[:n]
    big = sp[:, 2] > SMALL_SPLIT_CHUNKS
    order = torch.argsort((~big).to(torch.int8), stable=True)
    direction.splits[:n] = sp[order].clone()
    direction.n_split_big = int(big.sum().item())
    return direction.n_split_big


def _schedule(rowptr: torch.Tensor, N: int, E: int, chunk: int, side_split: int, row_mask, stream: int):
    lib = _ffi.load()
    dev = rowptr.device
    bytes_ = _ffi._sz(0)
    _ffi.check(lib.lgcn_schedule_workspace_size(E, N, chunk, bytes_), "lgcn_schedule_workspace_size")
    ws2 = torch.empty(max(1, bytes_.value), dtype=torch.uint8, device=dev)
    cap = N + E // chunk + 1
    items = torch.empty((cap, 2), dtype=torch.int64, device=dev)
    splits = torch.empty((max(N, 1), 4), dtype=torch.int32, device=dev)
    counts = torch.zeros(3, dtype=torch.int64, device=dev)
    _ffi.check(lib.lgcn_schedule_build(rowptr.data_ptr(), N, E, chunk, side_split, _ffi.ptr(row_mask), items.data_ptr(),
                                       cap, splits.data_ptr(), splits.shape[0], counts.data_ptr(), ws2.data_ptr(),
                                       ws2.numel(), stream), "lgcn_schedule_build")
    n_items, n_splits, n_partials = (int(v) for v in counts.cpu().tolist())
    return items, splits, n_items, n_splits, n_partials


def segment_directions(keys: torch.Tensor, N: int, chunk: int = DEFAULT_CHUNK, row_mask: torch.Tensor | None = None):
    """Plans for summing rows C[j] into output row keys[j] (j = 0..M-1) with lgcn_spmm, weight 1,
    in j order within a row: (dense: every row scheduled, for a SCALE/STORE pass that also writes
    the empty rows; sparse: only rows with a contribution, for an ADD pass; with row_mask also
    masked: every masked row). Built once per Cluster-GCN batch for its fixed (user, positive)
    gradient rows."""
    lib = _ffi.load()
    dev = keys.device
    M = keys.numel()
    stream = _ffi.stream_of(dev)
    # lgcn_csr_build range-checks `other` (= the contribution index) against its node count too,
    # so build over max(N, M) rows; rows >= N stay empty and are sliced off
    Nb = max(N, M)
    bytes_ = _ffi._sz(0)
    _ffi.check(lib.lgcn_csr_workspace_size(M, Nb, bytes_), "lgcn_csr_workspace_size")
    ws = torch.empty(max(1, bytes_.value), dtype=torch.uint8, device=dev)
    rowptr_b = torch.empty(Nb + 1, dtype=torch.int64, device=dev)
    col = torch.empty(M, dtype=torch.int32, device=dev)
    eid = torch.empty(M, dtype=torch.int32, device=dev)
    err = torch.zeros(1, dtype=torch.int64, device=dev)
    other = torch.arange(M, dtype=torch.int64, device=dev)
    _ffi.check(lib.lgcn_csr_build(keys.data_ptr(), other.data_ptr(), M, Nb, rowptr_b.data_ptr(), col.data_ptr(),
                                  eid.data_ptr(), err.data_ptr(), ws.data_ptr(), ws.numel(), stream), "lgcn_csr_build")
    rowptr = rowptr_b[: N + 1].contiguous()
    val = torch.ones(M, dtype=torch.float32, device=dev)
    mask = (rowptr[1:] > rowptr[:-1]).to(torch.uint8)
    sd_ = _schedule(rowptr, N, M, chunk, 0, None, stream)
    dense = CsrDirection(rowptr, col, eid, val, *sd_, chunk, _block_split_for(sd_[1], sd_[3]))
    ss_ = _schedule(rowptr, N, M, chunk, 0, mask, stream)
    sparse = CsrDirection(rowptr, col, eid, val, *ss_, chunk, _block_split_for(ss_[1], ss_[3]))
    if int(err.item()):
        raise IndexError("segment keys out of range")
    if row_mask is None:
        return dense, sparse
    # every row of row_mask (0 where it has no contribution), e.g. a batch's touched rows
    sm_ = _schedule(rowptr, N, M, chunk, 0, row_mask, stream)
    masked = CsrDirection(rowptr, col, eid, val, *sm_, chunk, _block_split_for(sm_[1], sm_[3]))
    return dense, sparse, masked


def _build_direction(key: torch.Tensor, other: torch.Tensor, N: int, chunk: int, side_split: int,
                     dis: torch.Tensor | None, stream: int, row_mask: torch.Tensor | None = None) -> tuple[CsrDirection, torch.Tensor, int]:
    lib = _ffi.load()
    dev = key.device
    E = key.numel()
    bytes_ = _ffi._sz(0)
    _ffi.check(lib.lgcn_csr_workspace_size(E, N, bytes_), "lgcn_csr_workspace_size")
    ws = torch.empty(max(1, bytes_.value), dtype=torch.uint8, device=dev)
    rowptr = torch.empty(N + 1, dtype=torch.int64, device=dev)
    col = torch.empty(E, dtype=torch.int32, device=dev)
    eid = torch.empty(E, dtype=torch.int32, device=dev)
    err = torch.zeros(1, dtype=torch.int64, device=dev)
    _ffi.check(lib.lgcn_csr_build(_ffi.ptr(key), _ffi.ptr(other), E, N, rowptr.data_ptr(), col.data_ptr(),
                                  eid.data_ptr(), err.data_ptr(), ws.data_ptr(), ws.numel(), stream),
               "lgcn_csr_build")
    if dis is None:
        dis = torch.empty(N, dtype=torch.float32, device=dev)
        _ffi.check(lib.lgcn_inv_sqrt_degree(rowptr.data_ptr(), N, dis.data_ptr(), stream), "lgcn_inv_sqrt_degree")
    val = torch.empty(E, dtype=torch.float32, device=dev)
    _ffi.check(lib.lgcn_edge_norm(rowptr.data_ptr(), col.data_ptr(), N, E, dis.data_ptr(), val.data_ptr(), stream),
               "lgcn_edge_norm")

    _ffi.check(lib.lgcn_schedule_workspace_size(E, N, chunk, bytes_), "lgcn_schedule_workspace_size")
    ws2 = torch.empty(max(1, bytes_.value), dtype=torch.uint8, device=dev)
    cap = N + E // chunk + 1
    items = torch.empty((cap, 2), dtype=torch.int64, device=dev)
    splits = torch.empty((max(N, 1), 4), dtype=torch.int32, device=dev)
    counts = torch.zeros(3, dtype=torch.int64, device=dev)
    _ffi.check(lib.lgcn_schedule_build(rowptr.data_ptr(), N, E, chunk, side_split, _ffi.ptr(row_mask), items.data_ptr(), cap, splits.data_ptr(),
                                       splits.shape[0], counts.data_ptr(), ws2.data_ptr(), ws2.numel(), stream),
               "lgcn_schedule_build")
    # one host read-back per plan: ids check + schedule sizes (the launches need them)
    host = torch.cat([counts, err]).cpu()
    n_items, n_splits, n_partials, n_bad = (int(v) for v in host.tolist())
    del ws, ws2
    # touched-only (Cluster-GCN batch) plans: short chunks, few per split row -> one launch per layer
    return CsrDirection(rowptr, col, eid, val, items, splits, n_items, n_splits, n_partials, chunk,
                        row_mask is not None and _block_split_for(splits, n_splits)), dis, n_bad


class PropagationPlan:
    """Forward (+ lazily transposed) plan for one edge set over N = num_users + num_items nodes."""

    def __init__(self, edge_index: torch.Tensor, num_nodes: int, chunk: int = DEFAULT_CHUNK, side_split: int = 0,
                 touched_only: bool = False):
        """touched_only: schedule only rows incident to an edge of this edge set (both directions);
        rows outside are never written by a propagation over this plan. ``touched`` (uint8[N])
        marks them. Used by the sparse Cluster-GCN batch step (lgcn_amd.train_step)."""
        _ffi.require_device(edge_index, "PropagationPlan")
        if edge_index.dim() != 2 or edge_index.shape[0] != 2:
            raise ValueError(f"edge_index must be [2, E], got {tuple(edge_index.shape)}")
        if edge_index.dtype != torch.int64:
            raise TypeError(f"edge_index must be int64 (torch.long), got {edge_index.dtype}")
        self.num_nodes = int(num_nodes)
        self.num_edges = int(edge_index.shape[1])
        self.chunk = int(chunk)
        self.side_split = int(side_split)
        self.device = edge_index.device
        self._src = edge_index[0].contiguous()
        self._dst = edge_index[1].contiguous()
        stream = _ffi.stream_of(self.device)
        self.touched = None
        if touched_only:
            t = torch.zeros(self.num_nodes, dtype=torch.uint8, device=self.device)
            if self.num_edges:
                if int(edge_index.min()) < 0 or int(edge_index.max()) >= self.num_nodes:
                    raise IndexError(f"edge_index holds node ids outside [0, {self.num_nodes})")
                t[self._src] = 1
                t[self._dst] = 1
            self.touched = t
        # forward: rows = targets (PyG flow source_to_target aggregates at edge_index[1])
        self.fwd, self.dis, bad = _build_direction(self._dst, self._src, self.num_nodes, self.chunk,
                                                 self.side_split, None, stream, self.touched)
        if bad:
            raise IndexError(f"edge_index holds {bad} edge(s) with a node id outside [0, {self.num_nodes})")
        self._bwd: CsrDirection | None = None
        self._sched: dict = {}

    def schedule(self, which: str, d: int):
        """The direction ('fwd' or 'bwd') to propagate rows of width d with: the source-sliced
        schedule (lgcn_amd.sliced) when slice_bytes_for(N, d) enables it for this plan, else the
        plain CsrDirection. Built once per (direction, d)."""
        key = (which, int(d))
        if key in self._sched:
            return self._sched[key]
        direction = self.fwd if which == "fwd" else self.bwd
        out = direction
        sb = 0 if self.touched is not None else slice_bytes_for(self.num_nodes, d)
        if sb and self.num_edges:
            from .sliced import build_sliced, slice_bounds

            bounds = slice_bounds(self.num_nodes, self.side_split, d, sb)
            # the running sums cost ~2 row passes per slice: worth it only for dense enough graphs
            # (C2: 112 edges per row; a 5 % validation edge set, ~6, is faster unsliced)
            from . import tuning

            forced = tuning.get().slice_mb is not None
            if forced or self.num_edges >= 8 * (len(bounds) - 1) * self.num_nodes:
                out = build_sliced(direction, self.num_nodes, bounds, sliced_chunk(direction.chunk)) or direction
        self._sched[key] = out
        return out

    @property
    def bwd(self) -> CsrDirection:
        """Transposed plan (rows = sources) for the autograd backward; weights reuse the
        forward in-degree normalisation, so val_T[q] == val[edge] exactly."""
        if self._bwd is None:
            stream = _ffi.stream_of(self.device)
            self._bwd, _, _ = _build_direction(self._src, self._dst, self.num_nodes, self.chunk,
                                              self.side_split, self.dis, stream, self.touched)
        return self._bwd

    def nbytes(self) -> int:
        tot = 0
        for d in (self.fwd, self._bwd):
            if d is None:
                continue
            for t in (d.rowptr, d.col, d.eid, d.val, d.items, d.splits):
                tot += t.numel() * t.element_size()
        return tot + self.dis.numel() * 4


class PlanCache:
    """Plans keyed by the edge_index's content (lgcn_amd._cache: the tensor object itself while it
    lives unmodified, else a digest of its bytes) plus (num_nodes, side_split): a tensor modified in
    place through torch (which bumps its version counter) is rehashed, and a loader that collates a
    new tensor of the same edges each epoch reuses its plan. Writes torch's counter does not see
    (through numpy, .data, DLPack or a raw pointer) leave the old key: hand over a new tensor object
    then, or call lgcn_amd._cache.forget(t). Least recently used plans are evicted beyond
    max_entries."""

    def __init__(self, max_entries: int = 1024, chunk: int = DEFAULT_CHUNK):
        from ._cache import ContentLRU

        self.max_entries = max_entries
        self.chunk = chunk
        self._entries = ContentLRU(max_entries)

    def get(self, edge_index: torch.Tensor, num_nodes: int, side_split: int = 0) -> PropagationPlan:
        return self._entries.get(edge_index, lambda: PropagationPlan(edge_index, num_nodes, self.chunk, side_split),
                                 extra=(int(num_nodes), int(side_split)))

    def clear(self) -> None:
        self._entries.clear()

    def __len__(self) -> int:
        return len(self._entries)
