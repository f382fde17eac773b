"""Probe: what one combine launch of the reduce-mode rank step costs, and why. For a
grid's heaviest row group, after one pair item pass, times lgcn_spmm_pair's combine half alone
(HIP events, 50 launches) over: both passes' split rows (the production launch), only the big
rows (> 16 chunks, one workgroup each), only the small rows (one lane group each), and one split
row (the launch's fixed cost).
python tools/combine_probe.py [--grids 4x2,8x1]"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "movie-recommender-system-with-gnns_amd"))

from lgcn_amd import _ffi, synth  # noqa: E402
from lgcn_amd.sharded import ReducePlan, ShardGrid, UserShards  # noqa: E402


def passes(rp, x0u, part, x0i, acc, y):
    N, U, d = rp.shards.N, rp.shards.U, rp.d

    def pass_of(direction, x, y_, a, mode):
        return _ffi.Pass(direction.items.data_ptr(), direction.n_items, direction.splits.data_ptr(),
                         direction.n_splits, direction.col.data_ptr(), direction.val.data_ptr(),
                         _ffi.ptr(x[0]), _ffi.ptr(x[1]), x[2], None, None, N, _ffi.ptr(y_), _ffi.ptr(a[0]),
                         _ffi.ptr(a[1]), a[2], _ffi.ptr(rp._part(direction, d)), mode, 1.0, 1.0,
                         n_split_big=direction.n_split_big)

    pa = pass_of(rp.partial, (x0u, part, U), None, (part, part, U), _ffi.EPI_STORE)
    pb = pass_of(rp.users, (x0i, x0i, U), y, acc, _ffi.EPI_ADD)
    return pa, pb


def restrict(p, direction, which):
    """a copy of Pass p over a subset of its split rows (they are ordered big-first)."""
    q = _ffi.Pass()
    ctypes.memmove(ctypes.byref(q), ctypes.byref(p), ctypes.sizeof(p))
    nb = direction.n_split_big
    if which == "big":
        q.n_splits = nb
    elif which == "small":
        q.splits = p.splits + nb * 16  # lgcn_split_t: 16 bytes
        q.n_splits = p.n_splits - nb
        q.n_split_big = 0
    elif which == "one":
        q.n_splits, q.n_split_big = 1, 0
        q.splits = p.splits + (p.n_splits - 1) * 16
    return q


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grids", default="4x2,8x1")
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda")
    g = synth.ml25m_shaped(seed=0)
    U, I, N = g.num_users, g.num_items, g.num_nodes
    ei = torch.from_numpy(g.edge_index).to(dev)
    deg = np.bincount(g.edge_index[1], minlength=N)
    d_full = 64
    gen = torch.Generator(device=dev).manual_seed(0)
    uw = torch.randn(U, d_full, device=dev, generator=gen) * 0.01
    iw = torch.randn(I, d_full, device=dev, generator=gen) * 0.01
    lib = _ffi.load()
    s = _ffi.stream_of(dev)
    for spec in args.grids.split(","):
        R, F = (int(v) for v in spec.split("x"))
        grid = ShardGrid.build(R * F, 0, d_full, R, F)
        c0, c1 = grid.cols
        d = c1 - c0
        shards = UserShards.build(deg, U, R)
        for gr in sorted({0, R - 1}):
            rp = ReducePlan(ei, shards, gr, d)
            x0u, x0i = uw[:, c0:c1].contiguous(), iw[:, c0:c1].contiguous()
            part = torch.zeros((rp.I_pad, d), device=dev)
            acc = (torch.zeros((U, d), device=dev), None, N)
            y = torch.empty((U, d), device=dev)
            pa, pb = passes(rp, x0u, part, x0i, acc, y)
            _ffi.check(lib.lgcn_spmm_pair(ctypes.byref(pa), ctypes.byref(pb), N, d, 1, s), "items")
            st = {}
            for which in ("all", "big", "small", "one", "items"):
                qa = pa if which in ("all", "items") else restrict(pa, rp.partial, which)
                qb = pb if which in ("all", "items") else restrict(pb, rp.users, which)
                what = 1 if which == "items" else 2
                for _ in range(3):
                    _ffi.check(lib.lgcn_spmm_pair(ctypes.byref(qa), ctypes.byref(qb), N, d, what, s), which)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(args.reps):
                    _ffi.check(lib.lgcn_spmm_pair(ctypes.byref(qa), ctypes.byref(qb), N, d, what, s), which)
                e1.record()
                torch.cuda.synchronize()
                st[which] = e0.elapsed_time(e1) / args.reps * 1e3
            sp_a = rp.partial.splits[:rp.partial.n_splits, 2].cpu().numpy()
            sp_b = rp.users.splits[:rp.users.n_splits, 2].cpu().numpy()
            print(f"grid {spec} g={gr} d={d}: split rows partial {sp_a.size} (big {rp.partial.n_split_big}, max "
                  f"{sp_a.max()} chunks), users {sp_b.size} (big {rp.users.n_split_big}, max {sp_b.max()}); "
                  + ", ".join(f"{k} {v:.2f} us" for k, v in st.items()), flush=True)
            del rp


if __name__ == "__main__":
    main()
