"""Source-sliced propagation schedule: every layer is issued as one lgcn_spmm_run launch per
slice of the SOURCE id range, in ascending source order, so all XCDs gather from one slice of
x at a time — a slice small enough to stay in each XCD's 4 MB L2 — instead of from the whole
table. A row's CSR edges are sorted by source (the coalesced edge order), so its segments in
successive slices are successive runs of its edge list: the row's sum continues through the
running buffer from launch to launch and stays ONE sequential chain in CSR order — the same
arithmetic as CPU scatter_add_ (and as the unsplit rows of the default schedule).
Rows with a segment longer than ``chunk`` (hubs) are cut into chunks whose partials the combine
pass adds after the last slice (as the default schedule does for its split rows).

Built on the device from a direction's CSR with torch ops (once per edge set).
"""
from __future__ import annotations

import dataclasses

import torch

from . import _ffi
from .plan import CsrDirection

ITEM_FIRST = 0x20000000
ITEM_LAST = 0x40000000


@dataclasses.dataclass
class SlicedDirection:
    base: CsrDirection
    launches: list          # [(items int64 [n, 2] (lgcn_item_t), n)] in ascending source-slice order
    splits: torch.Tensor    # int32 [n_splits, 4] (lgcn_split_t) for hub rows
    n_splits: int
    n_partials: int
    bounds: list            # source-id slice boundaries

    @property
    def col(self):
        return self.base.col

    @property
    def val(self):
        return self.base.val


def slice_bounds(N: int, U: int, d: int, slice_bytes: int) -> list[int]:
    """Boundaries over [0, N): the user range and the item range each cut into slices of about
    slice_bytes of fp32 rows of width d."""
    out = [0]
    U = min(max(int(U), 0), N)
    for lo, hi in ((0, U), (U, N)):
        n = hi - lo
        if n <= 0:
            continue
        k = max(1, -(-n * d * 4 // slice_bytes))
        out += [lo + (n * i) // k for i in range(1, k)] + [hi]
    return sorted(set(out))


def build_sliced(f: CsrDirection, N: int, bounds: list[int], chunk: int = 256) -> SlicedDirection | None:
    """None when some row's neighbours are not in ascending order (an uncoalesced edge_index):
    its slice segments would not be successive runs of its edge list, so the chain could not
    follow CSR order — the plain schedule is used then."""
    dev = f.rowptr.device
    rowptr = f.rowptr
    col = f.col.long()
    E = col.numel()
    S = len(bounds) - 1
    deg = rowptr[1:] - rowptr[:-1]
    row = torch.repeat_interleave(torch.arange(N, device=dev), deg)
    if E > 1 and bool(((col[1:] < col[:-1]) & (row[1:] == row[:-1])).any()):
        return None
    bnd = torch.tensor(bounds[1:-1], dtype=torch.long, device=dev)
    s_of = torch.bucketize(col, bnd, right=True)
    start = torch.ones(E, dtype=torch.bool, device=dev)
    if E > 1:
        start[1:] = (row[1:] != row[:-1]) | (s_of[1:] != s_of[:-1])
    seg_beg = torch.nonzero(start).squeeze(1)
    nseg = seg_beg.numel()
    seg_len = torch.diff(torch.cat([seg_beg, torch.tensor([E], device=dev)]))
    seg_row = row[seg_beg]
    seg_s = s_of[seg_beg]
    # hub rows: any segment longer than chunk -> chunked partials + combine
    hub = torch.zeros(N, dtype=torch.bool, device=dev)
    hub[seg_row[seg_len > chunk]] = True
    seg_hub = hub[seg_row]
    # row items (non-hub segments), with FIRST / LAST flags
    first_seg = torch.ones(nseg, dtype=torch.bool, device=dev)
    last_seg = torch.ones(nseg, dtype=torch.bool, device=dev)
    if nseg > 1:
        first_seg[1:] = seg_row[1:] != seg_row[:-1]
        last_seg[:-1] = seg_row[1:] != seg_row[:-1]
    keep = ~seg_hub
    r_beg, r_len, r_row, r_s = seg_beg[keep], seg_len[keep], seg_row[keep], seg_s[keep]
    r_flags = torch.where(first_seg[keep], ITEM_FIRST, 0) | torch.where(last_seg[keep], ITEM_LAST, 0)
    # empty non-hub rows: one flag-only item in slice 0 (its epilogue still runs)
    empty = torch.nonzero(deg == 0).squeeze(1)
    r_beg = torch.cat([r_beg, torch.zeros_like(empty)])
    r_len = torch.cat([r_len, torch.zeros_like(empty)])
    r_row = torch.cat([r_row, empty])
    r_s = torch.cat([r_s, torch.zeros_like(empty)])
    r_flags = torch.cat([r_flags, torch.full_like(empty, ITEM_FIRST | ITEM_LAST)])
    r_word = (r_len | r_flags) | (r_row << 32)
    # hub chunks: partial slots per hub row in CSR order
    hseg = torch.nonzero(seg_hub).squeeze(1)
    h_len = seg_len[hseg]
    nch = (h_len + chunk - 1) // chunk
    c_seg = torch.repeat_interleave(hseg, nch)
    c_first = torch.cumsum(nch, 0) - nch
    c_idx = torch.arange(c_seg.numel(), device=dev) - torch.repeat_interleave(c_first, nch)
    c_beg = seg_beg[c_seg] + c_idx * chunk
    c_len = torch.minimum(seg_len[c_seg] - c_idx * chunk, torch.tensor(chunk, device=dev))
    c_row = seg_row[c_seg]
    c_s = seg_s[c_seg]
    hub_rows = torch.nonzero(hub).squeeze(1)
    per_row = torch.bincount(c_row, minlength=N)
    pbeg_row = torch.cumsum(per_row, 0) - per_row
    # chunks are generated in CSR order, so rank within the row = position - first position
    first_pos = torch.full((N,), -1, dtype=torch.long, device=dev)
    pos = torch.arange(c_row.numel(), device=dev)
    if c_row.numel():
        first_pos.scatter_reduce_(0, c_row, pos, reduce="amin", include_self=False)
    c_slot = pbeg_row[c_row] + (pos - first_pos[c_row])
    c_word = (c_len & 0xFFFFFFFF) | ((-(c_slot) - 1) << 32)
    n_partials = int(per_row.sum())
    splits = torch.stack([hub_rows, pbeg_row[hub_rows], per_row[hub_rows], torch.zeros_like(hub_rows)], 1)
    splits = splits.to(torch.int32).contiguous()
    # per-slice launches, longest first
    all_beg = torch.cat([r_beg, c_beg])
    all_len = torch.cat([r_len, c_len])
    all_word = torch.cat([r_word, c_word])
    all_s = torch.cat([r_s, c_s])
    order = torch.argsort(all_s * (1 << 32) + (chunk * 64 - torch.clamp(all_len, max=chunk * 64)), stable=True)
    all_beg, all_word, all_s = all_beg[order], all_word[order], all_s[order]
    counts = torch.bincount(all_s, minlength=S).tolist()
    items = torch.stack([all_beg, all_word], 1).contiguous()
    launches, o = [], 0
    for c in counts:
        launches.append((items[o:o + c], c))
        o += c
    return SlicedDirection(f, launches, splits, int(hub_rows.numel()), n_partials, list(bounds))


def _tail(sd: SlicedDirection, N, d, x, e, acc, y, mode, div, mul, partial, stream):
    xl, xh, xs = x
    el, eh, es = e if e is not None else (None, None, N)
    al, ah, as_ = acc
    return (_ffi.ptr(sd.base.col), _ffi.ptr(sd.base.val), N, d, _ffi.ptr(xl), _ffi.ptr(xh), xs, _ffi.ptr(el),
            _ffi.ptr(eh), es, _ffi.ptr(y), _ffi.ptr(al), _ffi.ptr(ah), as_, _ffi.ptr(partial), mode, div, mul, stream)


def spmm_sliced(sd: SlicedDirection, N: int, d: int, x, e, acc, y, mode: int, div: float, mul: float,
                run: torch.Tensor, partial: torch.Tensor | None, stream: int, combine: bool = True,
                timer=None) -> None:
    """One layer over a sliced direction: one lgcn_spmm_run per slice, then the hub combine.
    timer (bench.py): a callable(d) -> context manager bracketing each slice launch."""
    lib = _ffi.load()
    tail = _tail(sd, N, d, x, e, acc, y, mode, div, mul, partial, stream)
    for items, n in sd.launches:
        if n == 0:
            continue
        if timer is not None:
            with timer(d):
                rc = lib.lgcn_spmm_run(items.data_ptr(), n, None, 0, *tail, run.data_ptr())
        else:
            rc = lib.lgcn_spmm_run(items.data_ptr(), n, None, 0, *tail, run.data_ptr())
        _ffi.check(rc, "lgcn_spmm_run")
    if combine:
        spmm_sliced_combine(sd, N, d, x, e, acc, y, mode, div, mul, partial, stream)


def spmm_sliced_combine(sd: SlicedDirection, N: int, d: int, x, e, acc, y, mode: int, div: float, mul: float,
                        partial: torch.Tensor | None, stream: int) -> None:
    if sd.n_splits:
        lib = _ffi.load()
        tail = _tail(sd, N, d, x, e, acc, y, mode, div, mul, partial, stream)
        _ffi.check(lib.lgcn_spmm_combine(None, 0, sd.splits.data_ptr(), sd.n_splits, *tail), "lgcn_spmm_combine")


def propagate_forward_sliced(user_w: torch.Tensor, item_w: torch.Tensor, sd: SlicedDirection, K: int) -> torch.Tensor:
    """out[N, d] = LightGCN final embedding over a sliced forward direction (K >= 1)."""
    import numpy as np

    U, d = user_w.shape
    I = item_w.shape[0]
    N = U + I
    dev = user_w.device
    stream = _ffi.stream_of(dev)
    out = torch.empty((N, d), dtype=torch.float32, device=dev)
    x0 = (user_w, item_w, U)
    div = float(K + 1)
    mul = float(np.float32(1.0 / (K + 1)))
    acc = (out, None, N)
    partial = torch.empty((sd.n_partials, d), dtype=torch.float32, device=dev) if sd.n_partials else None
    bufs = [torch.empty((N, d), dtype=torch.float32, device=dev) for _ in range(2)]
    if K == 1:
        spmm_sliced(sd, N, d, x0, x0, acc, None, _ffi.EPI_FINAL_E, div, mul, bufs[0], partial, stream)
        return out
    # layer outputs double as the running-sum buffers (a row's y is only final after its last item)
    spmm_sliced(sd, N, d, x0, x0, acc, bufs[0], _ffi.EPI_INIT, 1.0, 1.0, bufs[0], partial, stream)
    for k in range(2, K):
        src, dst = bufs[(k - 2) % 2], bufs[(k - 1) % 2]
        spmm_sliced(sd, N, d, (src, None, N), None, acc, dst, _ffi.EPI_ADD, 1.0, 1.0, dst, partial, stream)
    last = bufs[(K - 2) % 2]
    spmm_sliced(sd, N, d, (last, None, N), None, acc, None, _ffi.EPI_FINAL_ACC, div, mul, bufs[(K - 1) % 2], partial,
                stream)
    return out
