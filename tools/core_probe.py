"""Probe: how much of the C2 forward would a dense hub core on MFMA take off the gather path?

For each (Tu, Ti): the pairs between the Tu highest-degree users and the Ti highest-degree items
are removed from the C2 graph (both directions); the K=3 d=64 forward of the remaining sparse
graph is timed with the production plan, and a bf16 GEMM of the core's shape (A[Tu, Ti] x
Z[Ti, 3*64], both directions, hipBLASLt via torch) stands in for the MFMA pass. Timing only.
"""
from __future__ import annotations

import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "movie-recommender-system-with-gnns_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import lgcn_amd  # noqa: E402
from lgcn_amd import synth  # noqa: E402
from lgcn_amd.plan import DEFAULT_CHUNK, PropagationPlan  # noqa: E402


def timed(fn, n=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def main():
    dev = torch.device("cuda", 0)
    g = synth.ml25m_shaped()
    U, I, N = g.num_users, g.num_items, g.num_nodes
    src, dst = g.edge_index
    m = src < U
    du = np.bincount(src[m], minlength=U)
    di = np.bincount(dst[m] - U, minlength=I)
    ru = np.empty(U, np.int64)
    ru[np.argsort(-du, kind="stable")] = np.arange(U)
    ri = np.empty(I, np.int64)
    ri[np.argsort(-di, kind="stable")] = np.arange(I)
    us = np.where(m, src, dst)
    it = np.where(m, dst, src) - U
    gen = torch.Generator(device=dev).manual_seed(0)
    uw = (torch.randn(U, 64, device=dev, generator=gen) * 0.01).contiguous()
    iw = (torch.randn(I, 64, device=dev, generator=gen) * 0.01).contiguous()
    K = 3
    for Tu, Ti in [(0, 0), (8192, 1024), (16384, 1024), (16384, 2048), (32768, 1024), (32768, 2048),
                   (32768, 4096), (65536, 2048), (65536, 4096)]:
        core = (ru[us] < Tu) & (ri[it] < Ti)
        ei = torch.from_numpy(np.ascontiguousarray(g.edge_index[:, ~core])).to(dev)
        plan = PropagationPlan(ei, N, DEFAULT_CHUNK, side_split=U)
        with torch.no_grad():
            ms = timed(lambda: lgcn_amd.propagate_forward(uw, iw, plan, K))
        line = f"Tu {Tu:6d} Ti {Ti:5d} core pairs {core.sum() // 2 / 1e6:.2f}M sparse E {ei.shape[1] / 1e6:.2f}M " \
               f"sparse K=3 {ms:.3f} ms"
        if Tu:
            A = torch.zeros(Tu, Ti, dtype=torch.bfloat16, device=dev)
            At = torch.zeros(Ti, Tu, dtype=torch.bfloat16, device=dev)
            Zi = torch.randn(Ti, 192, device=dev).bfloat16()
            Zu = torch.randn(Tu, 192, device=dev).bfloat16()
            g1 = timed(lambda: A @ Zi)
            g2 = timed(lambda: At @ Zu)
            fl = 2 * Tu * Ti * 192
            line += f" | gemm u<-i {g1 * 1e3:.1f} us ({fl / g1 / 1e9:.0f} TF)  i<-u {g2 * 1e3:.1f} us " \
                    f"({fl / g2 / 1e9:.0f} TF)  K=3 total {(ms + 3 * (g1 + g2)):.3f} ms"
            del A, At, Zi, Zu
        print(line, flush=True)
        del plan, ei
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
