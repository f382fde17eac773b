"""lgcn_amd — MI355X-native LightGCN propagation (hand-written HIP kernels behind a C ABI).

Public pieces:
    PropagationPlan / PlanCache   device CSR + gcn_norm weights + load-balanced schedule
    lightgcn_propagate            K-layer propagation with autograd (one node)
    LGConv                        single-layer operator with the PyG LGConv call signature
    tuning / set_tuning           the process-wide schedule choices (no environment variables)
"""
from . import _ffi, tuning
from .tuning import set_tuning
from .plan import DEFAULT_CHUNK, CsrDirection, PlanCache, PropagationPlan
from .propagate import (LGConvFunction, LightGCNPropagation, lightgcn_propagate, propagate_backward,
                        propagate_forward, set_launch_timer)

import torch as _torch


class LGConv(_torch.nn.Module):
    """Parameter-free LightGCN layer, call-compatible with torch_geometric.nn.LGConv (PyG 2.4.0)
    as the reference uses it: ``LGConv()(x=Tensor[N,d], edge_index=LongTensor[2,E])``
    (reference models/light_gcn.py:24,33). gcn_norm is computed once per edge_index and cached."""

    def __init__(self, normalize: bool = True):
        super().__init__()
        if not normalize:
            raise NotImplementedError("LGConv(normalize=False) is not used by the reference and not provided")
        self.normalize = normalize
        self._plans = PlanCache(max_entries=64)

    def forward(self, x, edge_index, edge_weight=None):
        if edge_weight is not None:
            raise NotImplementedError("edge_weight is not used by the reference's LightGCN (models/light_gcn.py:33)")
        plan = self._plans.get(edge_index, x.shape[0])
        return LGConvFunction.apply(x, plan)

    def __repr__(self):
        return "LGConv()"


__all__ = ["DEFAULT_CHUNK", "CsrDirection", "PlanCache", "PropagationPlan", "LGConv", "LightGCNPropagation",
           "lightgcn_propagate", "propagate_forward", "propagate_backward", "set_launch_timer", "set_tuning",
           "tuning", "_ffi"]
