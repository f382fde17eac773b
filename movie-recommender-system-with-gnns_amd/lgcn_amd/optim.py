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
