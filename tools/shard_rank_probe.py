"""Probe: one rank's compute share of the sharded C2 forward (lgcn_amd.sharded) on one GPU, per
R x F grid, without the exchange (exchange=None): the time a rank spends in its kernels per K=3
step, to set against the all_gather volume per layer. python tools/shard_rank_probe.py"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "movie-recommender-system-with-gnns_amd"))

from lgcn_amd import synth  # noqa: E402
from lgcn_amd.sharded import RowShards, ShardedPlan, ShardGrid, propagate_forward_sharded  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grids", default="1x1,2x1,4x1,8x1,1x2,2x2,4x2,2x4")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--chunks", default="256")
    ap.add_argument("--plain", action="store_true", help="tuning slice_mb=0: the plain item schedule")
    ap.add_argument("--full-slices", action="store_true", help="R = 1 ranks keep the full width's slices")
    args = ap.parse_args()
    if args.plain:
        from lgcn_amd import tuning

        tuning.set_tuning(slice_mb=0.0)
    dev = torch.device("cuda")
    g = synth.ml25m_shaped(seed=0)
    U, I, N, E = g.num_users, g.num_items, g.num_nodes, g.num_edges
    ei = torch.from_numpy(g.edge_index).to(dev)
    deg = np.bincount(g.edge_index[1], minlength=N)
    K, d = 3, 64
    gen = torch.Generator(device=dev).manual_seed(0)
    uw = torch.randn(U, d, device=dev, generator=gen) * 0.01
    iw = torch.randn(I, d, device=dev, generator=gen) * 0.01
    for spec, chunk in [(sp, int(c)) for c in args.chunks.split(",") for sp in args.grids.split(",")]:
        R, F = (int(v) for v in spec.split("x"))
        grid = ShardGrid.build(R * F, 0, d, R, F)
        c0, c1 = grid.cols
        shards = RowShards.build(deg, U, R)
        times = []
        for gr in sorted({0, R - 1}):
            splan = ShardedPlan(ei, shards, gr, c1 - c0, chunk, slice_d=d if args.full_slices else None)
            x0p = shards.to_padded(uw[:, c0:c1].contiguous(), iw[:, c0:c1].contiguous())
            with torch.no_grad():
                for _ in range(3):
                    propagate_forward_sharded(x0p, splan, K, None)
                torch.cuda.synchronize()
                t = time.perf_counter()
                for _ in range(args.steps):
                    propagate_forward_sharded(x0p, splan, K, None)
                torch.cuda.synchronize()
            times.append((time.perf_counter() - t) / args.steps * 1e3)
            del splan, x0p
        xchg = (K - 1) * shards.NP * (c1 - c0) * 4 * (R - 1) / R
        print(f"grid {R}x{F} chunk {chunk}{' plain' if args.plain else ''}: rank compute {max(times):.3f} ms/step (row groups {sorted({0, R - 1})}: "
              f"{', '.join(f'{t:.3f}' for t in times)}); all_gather bytes received per rank per step "
              f"{xchg / 1e6:.1f} MB", flush=True)


if __name__ == "__main__":
    main()
