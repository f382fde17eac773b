"""K-layer LightGCN propagation on the MI355X kernels, with its autograd backward.

Forward (reference models/light_gcn.py:29-38, LGConv = PyG 2.4.0):
    x0 = cat(user_w, item_w)            -- never materialised: layer 1 reads both tables in place
    x_k = Â x_{k-1}, k = 1..K            -- one lgcn_spmm launch (+ split-row combine) per layer
    out = (sum_k x_k / (K+1)) * fp32(1/(K+1))   -- the layer-stack mean, fused into the epilogues
Backward: g = (dF * fp32(1/(K+1))) / (K+1) (MulBackward then MeanBackward), then
    G_K = g;  G_k = g + Âᵀ G_{k+1}  (k = K-1..0)  -- K launches over the transposed plan,
and G_0 is written straight into the two weight-gradient tables (the CatBackward split).
No intermediate x_k is saved: Â is linear, so the backward needs only the plan and dF.
"""
from __future__ import annotations


import numpy as np
import torch

from . import _ffi, tuning
from .plan import CsrDirection, PropagationPlan
from .sliced import SlicedDirection, spmm_sliced, spmm_sliced_combine

# Optional per-launch timing hook (bench.py): a callable(d, n_launches) -> context manager that
# records HIP events on the launching stream around n_launches item-pass launches.
_launch_timer = None


def set_launch_timer(timer) -> None:
    global _launch_timer
    _launch_timer = timer


def _f32(x: float) -> float:
    return float(np.float32(x))


def spmm(direction, N: int, d: int, x, e, acc, y, mode: int, div: float = 1.0, mul: float = 1.0,
         partial: torch.Tensor | None = None, stream: int | None = None) -> None:
    """One layer: one lgcn_spmm call over a CsrDirection, or the per-slice lgcn_spmm_run launches
    (+ hub combine) over a SlicedDirection. x / e / acc are split tables: (lo, hi, split) with
    hi=None for a single [N, d] table (split = N)."""
    lib = _ffi.load()
    if stream is None:
        stream = _ffi.stream_of(acc[0].device)
    if direction.n_partials > 0 and partial is None:
        partial = torch.empty((direction.n_partials, d), dtype=torch.float32, device=acc[0].device)
    if isinstance(direction, SlicedDirection):
        # the layer output doubles as the running-sum buffer (a row's y is final only after its
        # last item); the final-layer modes have no y, so they get a scratch one
        run = y if y is not None else torch.empty((N, d), dtype=torch.float32, device=acc[0].device)
        if _launch_timer is not None:
            # one bracket around the layer's slice launches (2 events per layer, not per launch)
            with _launch_timer(d, direction.n_launches):
                spmm_sliced(direction, N, d, x, e, acc, y, mode, div, mul, run, partial, stream, combine=False)
            spmm_sliced_combine(direction, N, d, x, e, acc, y, mode, div, mul, partial, stream)
        else:
            spmm_sliced(direction, N, d, x, e, acc, y, mode, div, mul, run, partial, stream)
        return
    xl, xh, xs = x
    el, eh, es = e if e is not None else (None, None, N)
    al, ah, as_ = acc
    if direction.block_split and direction.n_splits and d % 4 == 0 and d <= 1024 and (d & (d - 1)) == 0:
        # one launch: split rows summed by one workgroup each (bitwise the items + combine pair)
        rows, n_rows, chunks = direction.block_lists()
        args = (rows.data_ptr(), n_rows, direction.splits.data_ptr(), direction.n_splits,
                direction.col.data_ptr(), direction.val.data_ptr(), N, d,
                _ffi.ptr(xl), _ffi.ptr(xh), xs, _ffi.ptr(el), _ffi.ptr(eh), es,
                _ffi.ptr(y), _ffi.ptr(al), _ffi.ptr(ah), as_, None, mode, div, mul, stream, chunks.data_ptr())
        if _launch_timer is not None:
            with _launch_timer(d, 1):
                rc = lib.lgcn_spmm_blocksplit(*args)
        else:
            rc = lib.lgcn_spmm_blocksplit(*args)
        _ffi.check(rc, "lgcn_spmm_blocksplit")
        return
    args = (direction.items.data_ptr(), direction.n_items, direction.splits.data_ptr(), direction.n_splits,
            direction.col.data_ptr(), direction.val.data_ptr(), N, d,
            _ffi.ptr(xl), _ffi.ptr(xh), xs, _ffi.ptr(el), _ffi.ptr(eh), es,
            _ffi.ptr(y), _ffi.ptr(al), _ffi.ptr(ah), as_, _ffi.ptr(partial), mode, div, mul, stream)
    if _launch_timer is not None:
        # bracket the item pass (the dominant kernel) alone; the combine pass follows it
        with _launch_timer(d, 1):
            rc = lib.lgcn_spmm_items(*args)
        _ffi.check(rc, "lgcn_spmm_items")
        rc = lib.lgcn_spmm_combine(*args)
        _ffi.check(rc, "lgcn_spmm_combine")
        return
    _ffi.check(lib.lgcn_spmm(*args), "lgcn_spmm")


def _check_tables(user_w: torch.Tensor, item_w: torch.Tensor, plan: PropagationPlan) -> tuple[int, int, int]:
    for t, nm in ((user_w, "user_embedding.weight"), (item_w, "item_embedding.weight")):
        _ffi.require_device(t, nm)
        if t.dtype != torch.float32:
            raise TypeError(f"{nm} must be float32, got {t.dtype}")
        if not t.is_contiguous():
            raise ValueError(f"{nm} must be contiguous")
    U, d = user_w.shape
    I, d2 = item_w.shape
    if d != d2:
        raise ValueError(f"embedding widths differ: {d} vs {d2}")
    if U + I != plan.num_nodes:
        raise ValueError(f"plan was built for {plan.num_nodes} nodes, tables have {U + I}")
    if user_w.device != plan.device or item_w.device != plan.device:
        raise ValueError("embeddings and edge_index are on different devices")
    return U, I, d


def propagate_forward(user_w: torch.Tensor, item_w: torch.Tensor, plan: PropagationPlan, K: int) -> torch.Tensor:
    """out[N, d] = LightGCN final embedding (users first, then items)."""
    U, I, d = _check_tables(user_w, item_w, plan)
    N = U + I
    dev = user_w.device
    out = torch.empty((N, d), dtype=torch.float32, device=dev)
    stream = _ffi.stream_of(dev)
    x0 = (user_w, item_w, U)
    div = float(K + 1)
    mul = _f32(1.0 / (K + 1))
    acc = (out, None, N)
    if K == 0:
        lib = _ffi.load()
        _ffi.check(lib.lgcn_copy_scale(user_w.data_ptr(), item_w.data_ptr(), U, N, d, out.data_ptr(), div, mul, stream),
                   "lgcn_copy_scale")
        return out
    f = plan.schedule("fwd", d)
    if (K > 1 and isinstance(f, SlicedDirection) and tuning.get().slice_ride
            and d % 4 == 0 and d <= 1024 and (d & (d - 1)) == 0):
        from .sliced import ride_layout

        if ride_layout(f, U) is not None:
            _forward_sliced_ride(f, N, U, d, x0, acc, K, div, mul, stream)
            return out
    partial = torch.empty((f.n_partials, d), dtype=torch.float32, device=dev) if f.n_partials else None
    if K == 1:
        spmm(f, N, d, x0, x0, acc, None, _ffi.EPI_FINAL_E, div, mul, partial, stream)
        return out
    bufs = [torch.empty((N, d), dtype=torch.float32, device=dev) for _ in range(min(2, K - 1))]
    spmm(f, N, d, x0, x0, acc, bufs[0], _ffi.EPI_INIT, 1.0, 1.0, partial, stream)
    for k in range(2, K):
        src = bufs[(k - 2) % len(bufs)]
        dst = bufs[(k - 1) % len(bufs)]
        spmm(f, N, d, (src, None, N), None, acc, dst, _ffi.EPI_ADD, 1.0, 1.0, partial, stream)
    last = bufs[(K - 2) % len(bufs)]
    spmm(f, N, d, (last, None, N), None, acc, None, _ffi.EPI_FINAL_ACC, div, mul, partial, stream)
    return out


def _forward_sliced_ride(f, N: int, U: int, d: int, x0, acc, K: int, div: float, mul: float, stream: int) -> None:
    """propagate_forward over a sliced schedule with riding combines (K >= 2). Per layer the two
    slice groups run one after the other — user-table slices (writing item rows) and item-table
    slices (writing user rows), the group order alternating from layer to layer — and the split
    rows a group wrote are combined by extra workgroups of the NEXT group's first launch
    (lgcn_spmm_run_slices_ride): that launch gathers the other table of its layer and writes the
    other side's rows, so it never touches the rows, y or partial slots being combined. Partials
    alternate between two buffers by layer parity (a layer's first group writes the partial slots
    that the previous layer's split rows are being read from). The last group's split rows get a
    combine launch of their own. Each row: the slice launches and combine of propagate_forward,
    in the same order — bitwise its result."""
    import ctypes

    lib = _ffi.load()
    dev = acc[0].device
    r = f._ride
    S = len(f.launches)
    groups = {"u": (0, r["nu"]), "i": (r["nu"], S)}
    writes = {"u": "items", "i": "users"}
    parts = [torch.empty((f.n_partials, d), dtype=torch.float32, device=dev) if f.n_partials else None
             for _ in range(2)]
    bufs = [torch.empty((N, d), dtype=torch.float32, device=dev) for _ in range(min(2, K - 1))]
    scratch = torch.empty((N, d), dtype=torch.float32, device=dev)  # the last layer's running sums
    al, ah, as_ = acc
    offs = ctypes.addressof(f.host_offsets)

    def layer(k):
        if k == 1:
            return dict(x=x0, e=x0, y=bufs[0], mode=_ffi.EPI_INIT, div=1.0, mul=1.0, part=parts[1])
        x = (bufs[(k - 2) % len(bufs)], None, N)
        if k < K:
            return dict(x=x, e=None, y=bufs[(k - 1) % len(bufs)], mode=_ffi.EPI_ADD, div=1.0, mul=1.0,
                        part=parts[k % 2])
        return dict(x=x, e=None, y=None, mode=_ffi.EPI_FINAL_ACC, div=div, mul=mul, part=parts[k % 2])

    def ride_pass(side, lay):
        beg, n, nb = r[side]
        if n == 0:
            return None
        xl, xh, xs = lay["x"]
        el, eh, es = lay["e"] if lay["e"] is not None else (None, None, N)
        return _ffi.Pass(None, 0, f.splits.data_ptr() + 16 * beg, n, _ffi.ptr(f.base.col), _ffi.ptr(f.base.val),
                         _ffi.ptr(xl), _ffi.ptr(xh), xs, _ffi.ptr(el), _ffi.ptr(eh), es, _ffi.ptr(lay["y"]),
                         _ffi.ptr(al), _ffi.ptr(ah), as_, _ffi.ptr(lay["part"]), lay["mode"], lay["div"], lay["mul"],
                         n_split_big=nb)

    pending = None  # the split rows of the last group issued, with their layer's arguments
    if _launch_timer is not None:
        # one bracket around all K layers' slice launches (2 events per step; the last combine
        # launch below stays outside it), so launches x mean <= the step time by construction
        with _launch_timer(d, K * sum(1 for _, n in f.launches if n)):
            pending = _ride_layers(f, N, d, K, r, groups, writes, layer, ride_pass, scratch, acc, offs, stream, lib)
    else:
        pending = _ride_layers(f, N, d, K, r, groups, writes, layer, ride_pass, scratch, acc, offs, stream, lib)
    ride = ride_pass(*pending)
    if ride is not None:
        _ffi.check(lib.lgcn_spmm_pass(ctypes.byref(ride), N, d, 2, stream), "lgcn_spmm_pass (last combine)")


def _ride_layers(f, N, d, K, r, groups, writes, layer, ride_pass, scratch, acc, offs, stream, lib):
    """The K layers' slice-group launches of _forward_sliced_ride; returns the last group's pending
    split rows (combined by the caller's final launch)."""
    import ctypes

    al, ah, as_ = acc
    pending = None
    for k in range(1, K + 1):
        lay = layer(k)
        xl, xh, xs = lay["x"]
        el, eh, es = lay["e"] if lay["e"] is not None else (None, None, N)
        run = lay["y"] if lay["y"] is not None else scratch
        for grp in (("u", "i") if k % 2 == 1 else ("i", "u")):
            a, b = groups[grp]
            ride = ride_pass(*pending) if pending is not None else None
            args = (f.items.data_ptr(), ctypes.c_void_p(offs + 8 * a), b - a, _ffi.ptr(f.base.col),
                    _ffi.ptr(f.base.val), N, d, _ffi.ptr(xl), _ffi.ptr(xh), xs, _ffi.ptr(el), _ffi.ptr(eh), es,
                    _ffi.ptr(lay["y"]), _ffi.ptr(al), _ffi.ptr(ah), as_, _ffi.ptr(lay["part"]), lay["mode"],
                    lay["div"], lay["mul"], stream, run.data_ptr(),
                    ctypes.byref(ride) if ride is not None else None, 0)
            _ffi.check(lib.lgcn_spmm_run_slices_ride(*args), "lgcn_spmm_run_slices_ride")
            pending = (writes[grp], lay)
    return pending


def propagate_backward(dout: torch.Tensor, plan: PropagationPlan, U: int, K: int) -> tuple[torch.Tensor, torch.Tensor]:
    """(grad_user [U,d], grad_item [I,d]) of out = propagate_forward(...) given dout [N,d]."""
    dout = dout.contiguous()
    if dout.dtype != torch.float32:
        dout = dout.float()
    N, d = dout.shape
    I = N - U
    dev = dout.device
    stream = _ffi.stream_of(dev)
    lib = _ffi.load()
    grad_user = torch.empty((U, d), dtype=torch.float32, device=dev)
    grad_item = torch.empty((I, d), dtype=torch.float32, device=dev)
    div = float(K + 1)
    mul = _f32(1.0 / (K + 1))
    if K == 0:
        # d/dx0 of (x0/1)*1 is (dF*1)/1: the scale kernel writes straight into both grads
        _ffi.check(lib.lgcn_scale(dout.data_ptr(), grad_user.data_ptr(), U * d, mul, div, stream), "lgcn_scale")
        _ffi.check(lib.lgcn_scale(dout[U:].data_ptr(), grad_item.data_ptr(), I * d, mul, div, stream), "lgcn_scale")
        return grad_user, grad_item
    g = torch.empty((N, d), dtype=torch.float32, device=dev)
    _ffi.check(lib.lgcn_scale(dout.data_ptr(), g.data_ptr(), N * d, mul, div, stream), "lgcn_scale")
    b = plan.schedule("bwd", d)
    partial = torch.empty((b.n_partials, d), dtype=torch.float32, device=dev) if b.n_partials else None
    cur = g
    bufs = [torch.empty((N, d), dtype=torch.float32, device=dev) for _ in range(min(2, K - 1))]
    for step in range(K):
        last = step == K - 1
        if last:
            acc = (grad_user, grad_item, U)
        else:
            nxt = bufs[step % len(bufs)]
            acc = (nxt, None, N)
        spmm(b, N, d, (cur, None, N), (g, None, N), acc, None, _ffi.EPI_INIT, 1.0, 1.0, partial, stream)
        if not last:
            cur = nxt
    return grad_user, grad_item


def propagate_backward_seeded(grad_user: torch.Tensor, grad_item: torch.Tensor, plan: PropagationPlan, K: int) -> None:
    """In-place backward for the sparse batch step: on entry the two gradient tables hold the seed
    g = (dF * mul) / div for EVERY row; on exit they hold dL/dx0. Only the plan's scheduled rows
    change (with a touched-only plan, rows no batch edge reaches keep g, which is their exact
    gradient: every layer adds 0 to them)."""
    U, d = grad_user.shape
    I = grad_item.shape[0]
    N = U + I
    if K == 0:
        return
    dev = grad_user.device
    stream = _ffi.stream_of(dev)
    b = plan.schedule("bwd", d)
    partial = torch.empty((b.n_partials, d), dtype=torch.float32, device=dev) if b.n_partials else None
    g = (grad_user, grad_item, U)
    if K == 1:
        # the gather source must not alias the table being written
        src = torch.cat([grad_user, grad_item])
        spmm(b, N, d, (src, None, N), g, g, None, _ffi.EPI_INIT, 1.0, 1.0, partial, stream)
        return
    bufs = [torch.empty((N, d), dtype=torch.float32, device=dev) for _ in range(min(2, K - 1))]
    cur = g
    for step in range(K):
        last = step == K - 1
        acc = g if last else (bufs[step % len(bufs)], None, N)
        spmm(b, N, d, cur, g, acc, None, _ffi.EPI_INIT, 1.0, 1.0, partial, stream)
        cur = acc


class LightGCNPropagation(torch.autograd.Function):
    """autograd node for the whole K-layer propagation (one node instead of K LGConv nodes)."""

    @staticmethod
    def forward(ctx, user_w, item_w, plan: PropagationPlan, K: int):
        out = propagate_forward(user_w.detach(), item_w.detach(), plan, K)
        ctx.plan = plan
        ctx.K = K
        ctx.U = user_w.shape[0]
        return out

    @staticmethod
    def backward(ctx, dout):
        gu, gi = propagate_backward(dout, ctx.plan, ctx.U, ctx.K)
        return gu, gi, None, None


def lightgcn_propagate(user_w: torch.Tensor, item_w: torch.Tensor, plan: PropagationPlan, K: int) -> torch.Tensor:
    return LightGCNPropagation.apply(user_w, item_w, plan, K)


# ---- single-layer operator (the reference's LGConv()(x, edge_index) boundary) ----

def lgconv_forward(x: torch.Tensor, plan: PropagationPlan) -> torch.Tensor:
    _ffi.require_device(x, "LGConv")
    if x.dtype != torch.float32:
        raise TypeError(f"LGConv input must be float32, got {x.dtype}")
    x = x.contiguous()
    N, d = x.shape
    if N != plan.num_nodes:
        raise ValueError(f"x has {N} rows, plan has {plan.num_nodes} nodes")
    out = torch.empty_like(x)
    spmm(plan.schedule("fwd", d), N, d, (x, None, N), None, (out, None, N), None, _ffi.EPI_STORE)
    return out


def lgconv_backward(dy: torch.Tensor, plan: PropagationPlan) -> torch.Tensor:
    dy = dy.contiguous().float()
    N, d = dy.shape
    dx = torch.empty_like(dy)
    spmm(plan.schedule("bwd", d), N, d, (dy, None, N), None, (dx, None, N), None, _ffi.EPI_STORE)
    return dx


class LGConvFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, plan: PropagationPlan):
        ctx.plan = plan
        return lgconv_forward(x.detach(), plan)

    @staticmethod
    def backward(ctx, dy):
        return lgconv_backward(dy, ctx.plan), None
