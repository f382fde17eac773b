"""FusedAdam: the reference's clip_grad_norm_(max_norm=1) + optim.Adam(lr=1e-3) step
(reference utils/train_test.py:95-96,236) as two HIP launches (lgcn_grad_norm, lgcn_adam_step)
instead of ~20 PyTorch multi-tensor launches, with no host synchronisation.

Same hyper-parameters and update rule as torch.optim.Adam's defaults (betas (0.9, 0.999),
eps 1e-8, no weight decay, no amsgrad); bias corrections are computed in double on the host
from a Python step counter, as torch does when not capturable.
"""
from __future__ import annotations

import ctypes

import torch

from . import _ffi


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 max_grad_norm: float | None = None, keep_clipped_grad: bool = True, capturable: bool = False):
        """capturable=True keeps the step counter and bias corrections on the device
        (lgcn_adam_prologue), so the step can be captured in a hipGraph and replayed."""
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps))
        self.fused_clip_norm = max_grad_norm
        self.keep_clipped_grad = keep_clipped_grad
        self.capturable = capturable
        self.last_norm = None  # device tensor [total_norm, clip_coef] of the last clipped step
        self._norm_ws = None
        self._norm_out = None

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = _ffi.load()
        for group in self.param_groups:
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            for p in ps:
                _ffi.require_device(p, "FusedAdam")
                if p.dtype != torch.float32 or p.grad.dtype != torch.float32 or not p.is_contiguous() \
                        or not p.grad.is_contiguous():
                    raise TypeError("FusedAdam handles contiguous fp32 params and grads")
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
            if self.capturable and "dev_step" not in group:
                group["dev_step"] = torch.zeros(1, dtype=torch.float64, device=ps[0].device)
                group["dev_scalars"] = torch.zeros(2, dtype=torch.float32, device=ps[0].device)
            for i in range(0, len(ps), 8):
                self._step_chunk(lib, group, ps[i:i + 8], first=(i == 0))
        return loss

    def _step_chunk(self, lib, group, ps, first=True):
        dev = ps[0].device
        stream = _ffi.stream_of(dev)
        arr = (_ffi.AdamTensor * len(ps))()
        for k, p in enumerate(ps):
            st = self.state[p]
            arr[k] = _ffi.AdamTensor(p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(),
                                     st["exp_avg_sq"].data_ptr(), p.numel())
        clip_ptr = None
        if self.fused_clip_norm is not None:
            if self._norm_ws is None or self._norm_ws.device != dev:
                self._norm_ws = torch.empty(lib.lgcn_grad_norm_workspace_floats(), dtype=torch.float32, device=dev)
                self._norm_out = torch.empty(2, dtype=torch.float32, device=dev)
            out = self._norm_out
            _ffi.check(lib.lgcn_grad_norm(arr, len(ps), float(self.fused_clip_norm), self._norm_ws.data_ptr(),
                                          out.data_ptr(), stream), "lgcn_grad_norm")
            self.last_norm = out
            clip_ptr = out.data_ptr()  # kernel reads element [1]
        beta1, beta2 = group["betas"]
        st0 = self.state[ps[0]]
        # every param of a group advances together (as the reference's single-group Adam)
        step = st0["step"] + 1
        for p in ps:
            self.state[p]["step"] = step
        dev_scalars = None
        if self.capturable:
            if first:  # one device step per group
                _ffi.check(lib.lgcn_adam_prologue(group["dev_step"].data_ptr(), group["lr"], beta1, beta2,
                                                  group["dev_scalars"].data_ptr(), stream), "lgcn_adam_prologue")
            dev_scalars = ctypes.c_void_p(group["dev_scalars"].data_ptr())
            step_size, bc2_sqrt = 0.0, 1.0
        else:
            bc1 = 1 - beta1 ** step
            bc2 = 1 - beta2 ** step
            step_size, bc2_sqrt = -(group["lr"] / bc1), bc2 ** 0.5
        _ffi.check(lib.lgcn_adam_step(arr, len(ps), 1 - beta1, beta2, 1 - beta2, group["eps"], step_size,
                                      bc2_sqrt, ctypes.c_void_p(clip_ptr) if clip_ptr else None, dev_scalars,
                                      1 if self.keep_clipped_grad else 0, stream), "lgcn_adam_step")


class RowLazyAdam:
    """Adam (+ clip_grad_norm_(max_norm)) over the two embedding tables, row-lazy and exact:
    a row's missed zero-gradient steps are replayed (lgcn_row_adam) when the row is next touched,
    with the arithmetic and per-step constants of FusedAdam(capturable=True), so after flush()
    every row holds what FusedAdam would have produced; only the clip coefficient's last bits
    can differ (its norm sums the touched rows only — the other rows' gradient is 0 — in another
    order). Driven by lgcn_amd.train_step.FusedTrainStep(lazy=True) — on one GPU, or data
    parallel with a lgcn_amd.distributed.RowExchange (every rank steps the union of the ranks'
    rows); parameters are stale between steps until flush() (call it before reading them:
    evaluation, checkpoints)."""

    def __init__(self, user_w: torch.Tensor, item_w: torch.Tensor, lr: float = 1e-3, betas=(0.9, 0.999),
                 eps: float = 1e-8, max_grad_norm: float | None = 1.0, max_steps: int = 1 << 24):
        for t in (user_w, item_w):
            _ffi.require_device(t, "RowLazyAdam")
            if t.dtype != torch.float32 or not t.is_contiguous():
                raise TypeError("RowLazyAdam handles contiguous fp32 tables")
        self.uw, self.iw = user_w, item_w
        self.U, self.d = user_w.shape
        self.N = self.U + item_w.shape[0]
        self.lr, self.betas, self.eps, self.max_grad_norm = float(lr), betas, float(eps), max_grad_norm
        dev = user_w.device
        self.device = dev
        self.m = (torch.zeros_like(user_w), torch.zeros_like(item_w))
        self.v = (torch.zeros_like(user_w), torch.zeros_like(item_w))
        self.last = torch.zeros(self.N, dtype=torch.int32, device=dev)
        self.claim = torch.full((self.N,), -1, dtype=torch.int32, device=dev)
        self.step_dev = torch.zeros(1, dtype=torch.int64, device=dev)
        self.steps = 0  # host mirror of the completed steps
        self.max_steps = int(max_steps)
        # (step size, sqrt(1 - beta2^t), its reciprocal, 0) per step t (lgcn_adam_consts)
        self.consts = torch.empty((self.max_steps + 2, 4), dtype=torch.float32, device=dev)
        lib = _ffi.load()
        self.regenerate_consts()
        self.norm_ws = torch.empty(lib.lgcn_row_grad_norm_workspace_floats(), dtype=torch.float32, device=dev)
        self.last_norm = torch.zeros(2, dtype=torch.float32, device=dev)
        # gradient tables: rows outside a step's touched set are never written or read
        self.gu = torch.empty_like(user_w)
        self.gi = torch.empty_like(item_w)

    def reserve(self, steps: int) -> bool:
        """Make room for step constants up to `steps` (at least doubling); True if the constant
        table moved (hipGraphs captured over the old one must be recaptured). The new table is
        regenerated whole, from the current lr: call it only when every row is current (load /
        flush), or the replays of past steps would use the new constants."""
        if steps <= self.max_steps:
            return False
        self.max_steps = max(int(steps), 2 * self.max_steps)
        self.consts = torch.empty((self.max_steps + 2, 4), dtype=torch.float32, device=self.device)
        self.regenerate_consts()
        return True

    def regenerate_consts(self) -> None:
        """The per-step constants [1, max_steps + 1) from the current lr and betas."""
        lib = _ffi.load()
        _ffi.check(lib.lgcn_adam_consts(self.consts.data_ptr(), 1, self.max_steps + 1, self.lr, float(self.betas[0]),
                                        float(self.betas[1]), _ffi.stream_of(self.device)), "lgcn_adam_consts")

    def _tables(self, with_grad: bool):
        p = (self.uw.data_ptr(), self.iw.data_ptr())
        g = (self.gu.data_ptr(), self.gi.data_ptr()) if with_grad else (None, None)
        return (*p, *g, self.m[0].data_ptr(), self.m[1].data_ptr(), self.v[0].data_ptr(), self.v[1].data_ptr(),
                self.U, self.d)

    def _row_adam(self, rows_a, keys_b, off_b, first_b, skip_b, n_rows, clip, mode, reg=None):
        lib = _ffi.load()
        b1, b2 = self.betas
        na = rows_a.numel() if rows_a is not None else 0
        nb = keys_b.numel() if keys_b is not None else 0
        if reg is not None:  # the update over g + the step's reg rows (mode 1 / 3)
            _ffi.check(lib.lgcn_row_adam_reg(*self._tables(True), _ffi.ptr(rows_a), na, _ffi.ptr(keys_b), nb, off_b,
                                             _ffi.ptr(first_b), _ffi.ptr(skip_b), self.last.data_ptr(),
                                             self.step_dev.data_ptr(), self.consts.data_ptr(), 1 - b1, b2, 1 - b2,
                                             self.eps, _ffi.ptr(clip), mode, ctypes.byref(reg),
                                             _ffi.stream_of(self.device)), "lgcn_row_adam_reg")
            return
        _ffi.check(lib.lgcn_row_adam(*self._tables(mode in (1, 3)), _ffi.ptr(rows_a), na, _ffi.ptr(keys_b), nb, off_b,
                                     _ffi.ptr(first_b), _ffi.ptr(skip_b), n_rows, self.last.data_ptr(),
                                     self.claim.data_ptr(), self.step_dev.data_ptr(), self.consts.data_ptr(),
                                     1 - b1, b2, 1 - b2, self.eps, _ffi.ptr(clip), mode,
                                     _ffi.stream_of(self.device)), "lgcn_row_adam")

    def catch_up(self, rows_a: torch.Tensor | None, keys_b: torch.Tensor | None = None, off_b: int = 0,
                 first_b: torch.Tensor | None = None, skip_b: torch.Tensor | None = None) -> None:
        """Bring the listed rows (duplicates allowed; list b filtered by first_b, and by skip_b[row]
        == 0) up to the completed step count."""
        self._row_adam(rows_a, keys_b, off_b, first_b, skip_b, 0, None, 0)

    # --- the owner-sharded exchange's pieces (lgcn_amd.owner): the clip norm over every rank's rows
    def sqnorm_partials(self, keys_b: torch.Tensor, skip_b: torch.Tensor, partials: torch.Tensor) -> None:
        """Block partials of the sum of squares of the gradient rows keys_b[j] with !skip_b[row].
        partials must hold lgcn_row_grad_norm_workspace_floats() floats (the kernel writes that many)."""
        lib = _ffi.load()
        need = lib.lgcn_row_grad_norm_workspace_floats()
        if partials.numel() < need or not partials.is_contiguous() or partials.dtype != torch.float32:
            raise ValueError(f"sqnorm_partials: partials must be {need} contiguous fp32, got "
                             f"{partials.numel()} {partials.dtype}")
        _ffi.check(lib.lgcn_row_grad_sqnorm(self.gu.data_ptr(), self.gi.data_ptr(), self.U, self.d, None, 0,
                                            keys_b.data_ptr(), keys_b.numel(), 0, None, skip_b.data_ptr(),
                                            partials.data_ptr(), _ffi.stream_of(self.device)),
                   "lgcn_row_grad_sqnorm")

    def step_rows_with_partials(self, keys_b: torch.Tensor, first_b: torch.Tensor,
                                partials_all: torch.Tensor | None) -> None:
        """One Adam step on the list's first-occurrence rows, clipped by the norm finished from
        every rank's partials (partials_all, rank order; None without clipping)."""
        if self.steps + 1 > self.max_steps:
            raise RuntimeError(f"RowLazyAdam: more than max_steps={self.max_steps} steps")
        clip = None
        if self.max_grad_norm is not None:
            lib = _ffi.load()
            _ffi.check(lib.lgcn_row_grad_norm_finish(partials_all.data_ptr(), partials_all.numel(),
                                                     float(self.max_grad_norm), self.last_norm.data_ptr(),
                                                     self.step_dev.data_ptr(), _ffi.stream_of(self.device)),
                       "lgcn_row_grad_norm_finish")
            clip = self.last_norm
        self._row_adam(None, keys_b, 0, first_b, None, 0, clip, 1 if clip is None else 3)
        self.steps += 1

    def step_rows(self, rows_a: torch.Tensor | None, keys_b: torch.Tensor | None = None, off_b: int = 0,
                  first_b: torch.Tensor | None = None, skip_b: torch.Tensor | None = None,
                  gather_partials=None, reg: _ffi.RegRows | None = None) -> None:
        """One Adam step whose gradient (self.gu / self.gi) is zero outside the listed rows, which
        must be duplicate-free (first_b / skip_b filter list b): clip norm over them, then the
        update; rows not listed are deferred. gather_partials (column-sharded training: each rank
        holds some columns of every row): called with this rank's norm block partials, returns
        every rank's partials in rank order — the norm is finished over all of them.
        reg (lgcn_reg_rows_t): the gradient is g + the step's BPR reg rows, formed by the norm and
        the update from their occurrence counts (g itself is not written)."""
        if self.steps + 1 > self.max_steps:
            raise RuntimeError(f"RowLazyAdam: more than max_steps={self.max_steps} steps")
        lib = _ffi.load()
        clip = None
        if reg is not None and gather_partials is not None:
            raise ValueError("step_rows: reg rows are formed for whole rows (no column partials)")
        if self.max_grad_norm is not None and gather_partials is not None:
            na = rows_a.numel() if rows_a is not None else 0
            nb = keys_b.numel() if keys_b is not None else 0
            if getattr(self, "_partials", None) is None:
                self._partials = torch.empty(lib.lgcn_row_grad_norm_workspace_floats(), dtype=torch.float32,
                                             device=self.device)
            _ffi.check(lib.lgcn_row_grad_sqnorm(self.gu.data_ptr(), self.gi.data_ptr(), self.U, self.d,
                                                _ffi.ptr(rows_a), na, _ffi.ptr(keys_b), nb, off_b, _ffi.ptr(first_b),
                                                _ffi.ptr(skip_b), self._partials.data_ptr(),
                                                _ffi.stream_of(self.device)), "lgcn_row_grad_sqnorm")
            every = gather_partials(self._partials)
            _ffi.check(lib.lgcn_row_grad_norm_finish(every.data_ptr(), every.numel(), float(self.max_grad_norm),
                                                     self.last_norm.data_ptr(), self.step_dev.data_ptr(),
                                                     _ffi.stream_of(self.device)), "lgcn_row_grad_norm_finish")
            self._row_adam(rows_a, keys_b, off_b, first_b, skip_b, 0, self.last_norm, 3)
            self.steps += 1
            return
        if self.max_grad_norm is not None:
            na = rows_a.numel() if rows_a is not None else 0
            nb = keys_b.numel() if keys_b is not None else 0
            args = (self.gu.data_ptr(), self.gi.data_ptr(), self.U, self.d, _ffi.ptr(rows_a), na, _ffi.ptr(keys_b), nb,
                    off_b, _ffi.ptr(first_b), _ffi.ptr(skip_b), float(self.max_grad_norm), self.norm_ws.data_ptr(),
                    self.last_norm.data_ptr(), self.step_dev.data_ptr())
            if reg is not None:
                _ffi.check(lib.lgcn_row_grad_norm_reg(*args, ctypes.byref(reg), _ffi.stream_of(self.device)),
                           "lgcn_row_grad_norm_reg")
            else:
                _ffi.check(lib.lgcn_row_grad_norm(*args, _ffi.stream_of(self.device)), "lgcn_row_grad_norm")
            clip = self.last_norm
        # with the clip norm, its finishing launch also advances the device step counter (mode 3:
        # one launch fewer per step); without it the update advances it itself (mode 1)
        self._row_adam(rows_a, keys_b, off_b, first_b, skip_b, 0, clip, 1 if clip is None else 3, reg)
        self.steps += 1

    def flush(self) -> None:
        """Replay every row up to the completed step count (parameters are current after it)."""
        self._row_adam(None, None, 0, None, None, self.N, None, 2)

    def exp_avg(self) -> tuple[torch.Tensor, torch.Tensor]:
        return self.m

    def exp_avg_sq(self) -> tuple[torch.Tensor, torch.Tensor]:
        return self.v
