"""The Cluster-GCN training step without autograd: the reference's per-batch step
(reference utils/train_test.py:86-101: zero_grad, compute_embeddings, bpr_loss, backward,
clip_grad_norm_(1), Adam step) as a fixed sequence of HIP launches.

    out  = LightGCN forward over the batch edges       (lgcn_spmm x K, cached plan)
    neg  = torch.randint(0, I, (B,))                   (same draw as reference sample_negative)
    loss, per-triplet grad rows = lgcn_bpr_fused       (+ lgcn_bpr_loss)
    dF   = rows scattered in a fixed order             (lgcn_csr_build over the 3B keys + lgcn_segment_rows)
    grads = LightGCN backward of dF                    (lgcn_scale + lgcn_spmm x K, transposed plan)
          + reg-gradient rows                          (lgcn_segment_rows, add)
    [all_reduce grads over ranks]; FusedAdam (clip fused) or any torch optimizer

Per batch the (user, positive) triplet halves are a fixed function of the batch edges
(reference utils/helpers.py:98-99), so they are computed once and cached with the plan; only the
negatives are drawn each step. No host synchronisation happens inside a step.
"""
from __future__ import annotations

import weakref

import torch

from . import _ffi
from .propagate import propagate_backward, propagate_forward


class _BatchState:
    def __init__(self, model, edge_index: torch.Tensor, d: int):
        dev = edge_index.device
        U, I = model.num_users, model.num_items
        N = U + I
        self.plan = model.plan_for(edge_index)
        src, dst = edge_index[0], edge_index[1]
        self.users = src[src < U].contiguous()
        self.pos = (dst[dst >= U] - U).contiguous()
        if self.users.numel() != self.pos.numel():
            raise ValueError("batch is not a symmetric bipartite edge list: users and positives differ in count")
        B = self.B = int(self.users.numel())
        self.neg = torch.empty(B, dtype=torch.int64, device=dev)
        self.keys = torch.empty(3 * B, dtype=torch.int64, device=dev)
        self.keys[:B] = self.users
        self.keys[B:2 * B] = self.pos + U
        self.cf = torch.empty((3 * B, d), dtype=torch.float32, device=dev)
        self.cw = torch.empty((3 * B, d), dtype=torch.float32, device=dev)
        self.terms = torch.empty(2 * B, dtype=torch.float32, device=dev)
        self.loss = torch.empty(1, dtype=torch.float32, device=dev)
        self.rowptr = torch.empty(N + 1, dtype=torch.int64, device=dev)
        self.col = torch.empty(3 * B, dtype=torch.int32, device=dev)
        self.eid = torch.empty(3 * B, dtype=torch.int32, device=dev)
        self.err = torch.zeros(1, dtype=torch.int64, device=dev)
        lib = _ffi.load()
        nbytes = _ffi._sz(0)
        _ffi.check(lib.lgcn_csr_workspace_size(3 * B, N, nbytes), "lgcn_csr_workspace_size")
        self.ws = torch.empty(max(1, nbytes.value), dtype=torch.uint8, device=dev)
        self.plan.bwd  # build the transposed plan now (its build reads counts back once)


class FusedTrainStep:
    """Callable training step for a LightGCN model (models.light_gcn.LightGCN).

    step(batch) -> device loss tensor [1]: gradients, optional DP all-reduce, optimizer step.
    compute_grads(batch) -> loss: sets user/item_embedding.weight.grad only."""

    def __init__(self, model, optimizer, bpr_coeff: float = 5e-3, world: int = 1, max_entries: int = 4096):
        self.model = model
        self.optimizer = optimizer
        self.coeff = float(bpr_coeff)
        self.world = world
        self.max_entries = max_entries
        self._states: dict[int, tuple[weakref.ref, int, _BatchState]] = {}

    def state(self, edge_index: torch.Tensor) -> _BatchState:
        hit = self._states.get(id(edge_index))
        if hit is not None:
            ref, ver, st = hit
            if ref() is edge_index and ver == edge_index._version:
                return st
        st = _BatchState(self.model, edge_index, self.model.dim_h)
        self._states[id(edge_index)] = (weakref.ref(edge_index), edge_index._version, st)
        if len(self._states) > self.max_entries:
            for k in [k for k, (r, _, _) in self._states.items() if r() is None]:
                self._states.pop(k)
        return st

    def compute_grads(self, batch) -> torch.Tensor:
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
        with torch.no_grad():
            out = propagate_forward(uw.detach(), iw.detach(), st.plan, K)
            torch.randint(0, I, (B,), device=dev, out=st.neg)
            torch.add(st.neg, U, out=st.keys[2 * B:])
            _ffi.check(lib.lgcn_bpr_fused(out.data_ptr(), None, N, uw.data_ptr(), iw.data_ptr(), U, U,
                                          st.users.data_ptr(), st.pos.data_ptr(), st.neg.data_ptr(), B, d,
                                          self.coeff, st.cf.data_ptr(), st.cw.data_ptr(), st.terms.data_ptr(),
                                          stream), "lgcn_bpr_fused")
            _ffi.check(lib.lgcn_bpr_loss(st.terms.data_ptr(), B, d, self.coeff, st.loss.data_ptr(), stream),
                       "lgcn_bpr_loss")
            _ffi.check(lib.lgcn_csr_build(st.keys.data_ptr(), st.keys.data_ptr(), 3 * B, N, st.rowptr.data_ptr(),
                                          st.col.data_ptr(), st.eid.data_ptr(), st.err.data_ptr(), st.ws.data_ptr(),
                                          st.ws.numel(), stream), "lgcn_csr_build")
            dF = torch.empty((N, d), dtype=torch.float32, device=dev)
            _ffi.check(lib.lgcn_segment_rows(st.rowptr.data_ptr(), st.eid.data_ptr(), st.cf.data_ptr(), N, d,
                                             dF.data_ptr(), None, N, 0, stream), "lgcn_segment_rows")
            gu, gi = propagate_backward(dF, st.plan, U, K)
            _ffi.check(lib.lgcn_segment_rows(st.rowptr.data_ptr(), st.eid.data_ptr(), st.cw.data_ptr(), N, d,
                                             gu.data_ptr(), gi.data_ptr(), U, 1, stream), "lgcn_segment_rows")
        uw.grad = gu
        iw.grad = gi
        return st.loss

    def step(self, batch) -> torch.Tensor:
        loss = self.compute_grads(batch)
        if self.world > 1:
            from .distributed import allreduce_grads

            allreduce_grads([self.model.user_embedding.weight, self.model.item_embedding.weight], self.world)
        if getattr(self.optimizer, "fused_clip_norm", None) is None:
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), max_norm=1)
        self.optimizer.step()
        return loss
