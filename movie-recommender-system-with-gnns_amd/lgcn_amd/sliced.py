"""Source-sliced propagation schedule: every layer is issued as one lgcn_spmm_run launch per
slice of the SOURCE id range, in ascending source order, so all XCDs gather from one slice of
x at a time — a slice small enough to stay in each XCD's 4 MB L2 — instead of from the whole
table. A row's CSR edges are sorted by source (the coalesced edge order), so its segments in
successive slices are successive runs of its edge list: the row's sum continues through the
running buffer from launch to launch and stays ONE sequential chain in CSR order — the same
arithmetic as CPU scatter_add_ (and as the unsplit rows of the default schedule).
Rows with a segment longer than ``chunk`` (hubs) are cut into chunks whose partials the combine
pass adds after the last slice (as the default schedule does for its split rows).

Built on the device from a direction's CSR by lgcn_slice_schedule_build (csrc/lgcn_plan.hip),
once per (edge set, width).
"""
from __future__ import annotations

import dataclasses

import torch

from . import _ffi
from .plan import CsrDirection

MAX_SLICES = 250  # lgcn_slice_schedule_build keys carry the slice in 8 bits
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
    items: torch.Tensor = None       # all items, slice-major (launches are views of it)
    host_offsets: object = None      # ctypes int64[S+1]: slice s = items[off[s]:off[s+1]]

    @property
    def n_launches(self) -> int:
        return sum(1 for _, n in self.launches if n)

    @property
    def col(self):
        return self.base.col

    @property
    def val(self):
        return self.base.val


def slice_bounds(N: int, U: int, d: int, slice_bytes: int) -> list[int]:
    """Boundaries over [0, N): the user range and the item range each cut into slices of about
    slice_bytes of fp32 rows of width d (at most MAX_SLICES in all)."""
    out = [0]
    U = min(max(int(U), 0), N)
    for lo, hi in ((0, U), (U, N)):
        n = hi - lo
        if n <= 0:
            continue
        k = min(MAX_SLICES // 2, max(1, -(-n * d * 4 // slice_bytes)))
        if lo == U and U > 0 and n * d * 4 <= 2 * slice_bytes:
            # an item range of up to two slices stays whole: every user row then gets its sum in one
            # segment (no running-sum store and reload between item slices). C2 d=64 (15.1 MB at
            # 8 MB slices): 1.230-1.234 -> 1.224-1.226 ms per K=3 step, 3 interleaved pairs
            # (profiles/r04u_item_slice/)
            k = 1
        out += [lo + (n * i) // k for i in range(1, k)] + [hi]
    return sorted(set(out))


def build_sliced(f: CsrDirection, N: int, bounds: list[int], chunk: int = 256,
                 row_mask: torch.Tensor | None = None) -> SlicedDirection | None:
    """The sliced schedule of direction f (lgcn_slice_schedule_build, on the device). None when
    some row's neighbours are not in ascending order (an uncoalesced edge_index): its slice
    segments would not be successive runs of its edge list, so the chain could not follow CSR
    order — the plain schedule is used then. row_mask (uint8[N]): schedule only those rows."""
    import ctypes

    lib = _ffi.load()
    dev = f.rowptr.device
    E = f.col.numel()
    S = len(bounds) - 1
    stream = _ffi.stream_of(dev)
    nbytes, cap = _ffi._sz(0), ctypes.c_int64(0)
    _ffi.check(lib.lgcn_slice_schedule_workspace_size(E, N, S, chunk, ctypes.byref(nbytes), ctypes.byref(cap)),
               "lgcn_slice_schedule_workspace_size")
    ws = torch.empty(max(1, nbytes.value), dtype=torch.uint8, device=dev)
    items = torch.empty((cap.value, 2), dtype=torch.int64, device=dev)
    splits = torch.empty((max(N, 1), 4), dtype=torch.int32, device=dev)
    offsets = torch.empty(S + 1, dtype=torch.int64, device=dev)
    counts = torch.zeros(4, dtype=torch.int64, device=dev)
    bnd = torch.tensor(bounds, dtype=torch.int64, device=dev)
    _ffi.check(lib.lgcn_slice_schedule_build(f.rowptr.data_ptr(), _ffi.ptr(f.col), N, E, bnd.data_ptr(), S, chunk,
                                             _ffi.ptr(row_mask), items.data_ptr(), cap.value, offsets.data_ptr(), splits.data_ptr(),
                                             splits.shape[0], counts.data_ptr(), ws.data_ptr(), ws.numel(), stream),
               "lgcn_slice_schedule_build")
    host = torch.cat([counts, offsets]).cpu().tolist()  # one read-back per plan
    n_items, n_splits, n_partials, unsorted = host[:4]
    off = host[4:]
    del ws
    if unsorted:
        return None
    launches = [(items[off[s]:off[s + 1]], off[s + 1] - off[s]) for s in range(S)]
    return SlicedDirection(f, launches, splits, n_splits, n_partials, list(bounds), items,
                           (ctypes.c_int64 * (S + 1))(*off))


def _tail(sd: SlicedDirection, N, d, x, e, acc, y, mode, div, mul, partial, stream):
    xl, xh, xs = x
    el, eh, es = e if e is not None else (None, None, N)
    al, ah, as_ = acc
    return (_ffi.ptr(sd.base.col), _ffi.ptr(sd.base.val), N, d, _ffi.ptr(xl), _ffi.ptr(xh), xs, _ffi.ptr(el),
            _ffi.ptr(eh), es, _ffi.ptr(y), _ffi.ptr(al), _ffi.ptr(ah), as_, _ffi.ptr(partial), mode, div, mul, stream)


def spmm_sliced(sd: SlicedDirection, N: int, d: int, x, e, acc, y, mode: int, div: float, mul: float,
                run: torch.Tensor, partial: torch.Tensor | None, stream: int, combine: bool = True,
                timer=None) -> None:
    """One layer over a sliced direction: one item-pass launch per slice (all issued by one
    lgcn_spmm_run_slices call), then the hub combine. timer (bench.py): a callable(d) -> context
    manager bracketing the layer's slice launches."""
    lib = _ffi.load()
    if sd.n_launches:
        # every slice launch of the layer from one host call (lgcn_spmm_run_slices loops in C)
        tail = _tail(sd, N, d, x, e, acc, y, mode, div, mul, partial, stream)
        args = (sd.items.data_ptr(), sd.host_offsets, len(sd.launches), *tail, run.data_ptr())
        if timer is not None:
            with timer(d):
                rc = lib.lgcn_spmm_run_slices(*args)
        else:
            rc = lib.lgcn_spmm_run_slices(*args)
        _ffi.check(rc, "lgcn_spmm_run_slices")
    if combine:
        spmm_sliced_combine(sd, N, d, x, e, acc, y, mode, div, mul, partial, stream)


def spmm_sliced_combine(sd: SlicedDirection, N: int, d: int, x, e, acc, y, mode: int, div: float, mul: float,
                        partial: torch.Tensor | None, stream: int) -> None:
    if sd.n_splits:
        lib = _ffi.load()
        tail = _tail(sd, N, d, x, e, acc, y, mode, div, mul, partial, stream)
        _ffi.check(lib.lgcn_spmm_combine(None, 0, sd.splits.data_ptr(), sd.n_splits, *tail), "lgcn_spmm_combine")


def _bipartite(rowptr: torch.Tensor, col: torch.Tensor, U: int) -> bool:
    """Every edge joins a row < U and a row >= U (then user-table slices write only item rows and
    item-table slices only user rows — what the riding combine relies on)."""
    N = rowptr.numel() - 1
    if col.numel() == 0:
        return True
    deg = rowptr[1:] - rowptr[:-1]
    dst_user = torch.repeat_interleave(torch.arange(N, device=col.device) < U, deg)
    return bool(((col < U) != dst_user).all().item())


def ride_layout(sd: SlicedDirection, U: int) -> dict | None:
    """Prepare sd for the riding combine of the K-layer forward (lgcn_spmm_run_slices_ride): its
    split rows ordered users first, then items, each side big-first (<= 16-chunk rows packed one
    per lane group), and the slice groups: slices [0, nu) gather user rows (they write item rows),
    [nu, S) gather item rows (they write user rows). None when the bounds do not separate the two
    tables (one group: nothing to ride in). One host read-back per plan."""
    r = getattr(sd, "_ride", None)
    if r is not None:
        return r or None
    S = len(sd.launches)
    nu = sd.bounds.index(U) if U in sd.bounds else -1
    base = sd.base
    if nu <= 0 or nu >= S or not _bipartite(base.rowptr, base.col, U):
        sd._ride = {}
        return None
    from .plan import SMALL_SPLIT_CHUNKS

    n = sd.n_splits
    counts = (0, 0, 0, 0)
    if n:
        sp = sd.splits[:n]
        side = (sp[:, 0] >= U).to(torch.int64)
        small = (sp[:, 2] <= SMALL_SPLIT_CHUNKS).to(torch.int64)
        key = side * 2 + small
        order = torch.argsort(key, stable=True)
        sd.splits[:n] = sp[order].clone()
        counts = tuple(int(v) for v in torch.bincount(key, minlength=4).cpu().tolist())
    n_users = counts[0] + counts[1]
    sd._ride = {"nu": nu, "users": (0, n_users, counts[0]), "items": (n_users, counts[2] + counts[3], counts[2])}
    return sd._ride


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
