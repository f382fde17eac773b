"""Projection of the reduce-mode C2 grid (lgcn_amd.sharded, users sharded, item partials all-reduced
per layer) to a node of R x F GPUs, from one GPU: each piece of a rank's K=3 step is timed alone
(HIP events, the rank's own plans, the heavier of row groups 0 and R-1), then the step is replayed
as an event schedule with the per-layer all_reduce / last-layer reduce_scatter priced from a bus
bandwidth and a latency that this box cannot measure (one GPU per box). Two orders:

  overlapped: P_k (+ its combine) -> all_reduce_k starts; U_k (+ combine) waits for all_reduce_{k-1}
              (P_k needs U_{k-1}); all_reduce_k overlaps U_k and P_{k+1}.
  fused:      pair_k = P_k and U_k in one launch (+ one combine launch), then all_reduce_k; pair_{k+1}
              waits for it.

python tools/project_scale.py [--grids 8x1,4x2] [--busbw 100,150,200,300] [--lat-us 15]"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "movie-recommender-system-with-gnns_amd"))

from lgcn_amd import _ffi, synth  # noqa: E402
from lgcn_amd.sharded import ReducePlan, ShardGrid, UserShards  # noqa: E402


def timed(fn, reps=30):
    """mean ms of fn() over reps (events on the current stream, after 3 warm-ups)."""
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def pieces(rplan, x0u, x0i, d):
    """ms of: the partial pass, the user pass, their pair launch (items + combines) — each a
    middle-layer (ADD) launch set on layer-0-shaped tables."""
    U, dev = x0u.shape[0], x0u.device
    I_pad = rplan.I_pad
    part = torch.zeros((I_pad, d), device=dev)
    acc_u = torch.zeros((U, d), device=dev)
    y = torch.empty((U, d), device=dev)
    acc = (acc_u, torch.zeros((x0i.shape[0], d), device=dev), U)
    t_p = timed(lambda: rplan.run_partial(x0u, part))
    t_u = timed(lambda: rplan.run_users(x0i, None, acc, y, _ffi.EPI_ADD, 1.0, 1.0))
    t_pair = timed(lambda: rplan.run_pair(x0u, part, x0i, None, acc, y, _ffi.EPI_ADD, 1.0, 1.0))
    return t_p, t_u, t_pair


def simulate(K, t_p, t_u, t_pair, t_ar, t_rs, fused):
    """ms per K-layer step of one rank (compute on one stream, the collectives serialised on
    another); the final stack mean (a few us) is ignored."""
    if fused:
        t, ar_done = 0.0, 0.0
        for k in range(1, K + 1):
            t = max(t, ar_done) + t_pair
            ar_done = t + (t_ar if k < K else t_rs)
        return ar_done
    t, comm, ar_done = 0.0, 0.0, {0: 0.0}
    for k in range(1, K + 1):
        t += t_p  # P_k needs U_{k-1}: the compute stream is in order
        comm = max(comm, t) + (t_ar if k < K else t_rs)
        ar_done[k] = comm
        t = max(t, ar_done[k - 1]) + t_u  # U_k reads the items reduced one layer earlier
    return max(t, ar_done[K])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grids", default="8x1,4x2")
    ap.add_argument("--busbw", default="100,150,200,300")
    ap.add_argument("--lat-us", type=float, default=15.0)
    ap.add_argument("--one-gpu-ms", type=float, default=1.2205, help="the one-GPU K=3 step (round 4, profiles/r04zd_final)")
    args = ap.parse_args()
    dev = torch.device("cuda")
    g = synth.ml25m_shaped(seed=0)
    U, I, N = g.num_users, g.num_items, g.num_nodes
    ei = torch.from_numpy(g.edge_index).to(dev)
    deg = np.bincount(g.edge_index[1], minlength=N)
    K, d_full = 3, 64
    gen = torch.Generator(device=dev).manual_seed(0)
    uw = torch.randn(U, d_full, device=dev, generator=gen) * 0.01
    iw = torch.randn(I, d_full, device=dev, generator=gen) * 0.01
    for spec in args.grids.split(","):
        R, F = (int(v) for v in spec.split("x"))
        grid = ShardGrid.build(R * F, 0, d_full, R, F)
        c0, c1 = grid.cols
        d = c1 - c0
        shards = UserShards.build(deg, U, R)
        worst = None
        for gr in sorted({0, R - 1}):
            rplan = ReducePlan(ei, shards, gr, d)
            x0u, x0i = uw[:, c0:c1].contiguous(), iw[:, c0:c1].contiguous()
            p = pieces(rplan, x0u, x0i, d)
            worst = p if worst is None or sum(p) > sum(worst) else worst
            del rplan
        t_p, t_u, t_pair = worst
        mb = rplan_bytes = (-(-I // R) * R) * d * 4 / 1e6  # one item table (padded) of this rank's columns
        print(f"grid {R}x{F} (d={d}/rank): partial pass {t_p * 1e3:.1f} us, user pass {t_u * 1e3:.1f} us, "
              f"pair {t_pair * 1e3:.1f} us (vs {1e3 * (t_p + t_u):.1f} us apart); item table {mb:.1f} MB", flush=True)
        for bw in (float(v) for v in args.busbw.split(",")):
            # ring all_reduce: 2 (R-1)/R of the table over the bus bandwidth; reduce_scatter half of it
            t_ar = args.lat_us / 1e3 + 2 * (R - 1) / R * rplan_bytes / bw  # MB / (GB/s) = ms
            t_rs = args.lat_us / 1e3 + (R - 1) / R * rplan_bytes / bw
            o = simulate(K, t_p, t_u, t_pair, t_ar, t_rs, False)
            f = simulate(K, t_p, t_u, t_pair, t_ar, t_rs, True)
            c = 3 * (t_p + t_u)
            print(f"  busbw {bw:.0f} GB/s (+{args.lat_us:.0f} us): all_reduce {t_ar * 1e3:.0f} us; step overlapped "
                  f"{o:.3f} ms ({args.one_gpu_ms / o:.2f}x), fused {f:.3f} ms ({args.one_gpu_ms / f:.2f}x); compute "
                  f"alone {c:.3f} / {3 * t_pair:.3f} ms ({args.one_gpu_ms / c:.2f}x / {args.one_gpu_ms / (3 * t_pair):.2f}x)",
                  flush=True)


if __name__ == "__main__":
    main()
