"""Probe: one rank's compute share of the reduce-mode sharded C2 forward (lgcn_amd.sharded.
ReducePlan: users sharded, item partials all-reduced) on one GPU, per R x F grid, without the
all_reduce (a stand-in reducer that moves nothing): the time a rank spends in its kernels per K=3
step, next to the bytes a ring all_reduce of its item partials moves per rank.
python tools/reduce_rank_probe.py [--grids 2x1,4x1,8x1,2x2,4x2,2x4] [--orders overlapped,fused,fused-seq]
A +g suffix (fused+g, ...) captures the step in a hipGraph once and times its replays (no host
launch overhead). Eager orders also print the host's issue time per step (the Python loop before
the synchronize; the stand-in reducer issues no collectives).
An order suffixed -u (overlapped-u, fused-u) combines every split row with a workgroup of its own
(n_split_big = -1) instead of packing the <= 16-chunk ones one per lane group."""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "movie-recommender-system-with-gnns_amd"))

from lgcn_amd import synth  # noqa: E402
from lgcn_amd.sharded import ReducePlan, ShardGrid, UserShards, propagate_forward_reduced  # noqa: E402


class NoReduce:
    """The reducer's interface, moving nothing (the compute side alone)."""

    def __init__(self, R):
        self.R, self.bytes = R, 0

    def start(self, buf):
        self.bytes += int(2 * (self.R - 1) / self.R * buf.numel() * buf.element_size())
        return None

    def start_scatter(self, buf, out, rank):
        self.bytes += int((self.R - 1) / self.R * buf.numel() * buf.element_size())
        return None

    def wait(self, handle, device):
        pass


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grids", default="2x1,4x1,8x1,2x2,4x2,2x4")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--chunk", type=int, default=256)
    ap.add_argument("--orders", default="overlapped,fused,fused-seq")
    ap.add_argument("--rank-chunk", type=int, default=0, help="override lgcn_amd.plan.RANK_CHUNK (0: keep)")
    args = ap.parse_args()
    if args.rank_chunk:
        from lgcn_amd import plan as _plan

        _plan.RANK_CHUNK = args.rank_chunk
    dev = torch.device("cuda")
    g = synth.ml25m_shaped(seed=0)
    U, I, N = g.num_users, g.num_items, g.num_nodes
    ei = torch.from_numpy(g.edge_index).to(dev)
    deg = np.bincount(g.edge_index[1], minlength=N)
    K, d = 3, 64
    gen = torch.Generator(device=dev).manual_seed(0)
    uw = torch.randn(U, d, device=dev, generator=gen) * 0.01
    iw = torch.randn(I, d, device=dev, generator=gen) * 0.01
    for spec in args.grids.split(","):
        R, F = (int(v) for v in spec.split("x"))
        grid = ShardGrid.build(R * F, 0, d, R, F)
        c0, c1 = grid.cols
        shards = UserShards.build(deg, U, R)
        times, moved = {o: [] for o in args.orders.split(",")}, 0
        host = {o: [] for o in times}  # the host's issue time per step (eager orders)
        for gr in sorted({0, R - 1}):
            rplan = ReducePlan(ei, shards, gr, c1 - c0, args.chunk)
            x0u, x0i = uw[:, c0:c1].contiguous(), iw[:, c0:c1].contiguous()
            red = NoReduce(R)
            moved_per_step = 0
            for order in times:
                graph = order.endswith("+g")
                base = order[:-2] if graph else order
                fused = base.startswith("fused")
                unpacked = base.endswith("-u")
                nb = {}
                for dr in (rplan.users, rplan.partial):
                    nb[id(dr)] = dr.n_split_big
                    if unpacked:
                        dr.n_split_big = -1
                # fused-seq: the pair launch without its XCD-split block mapping (pair_xcds_a=0);
                # fusedN: pass a (the item partials) on N of the 8 XCDs
                from lgcn_amd import tuning

                tuning.set_tuning(pair_xcds_a=0 if order == "fused-seq" else
                                  int(order[5:]) if order[5:].isdigit() else 4)
                with torch.no_grad():
                    for _ in range(3):
                        propagate_forward_reduced(x0u, x0i, rplan, K, red, fused=fused)
                    torch.cuda.synchronize()
                    red.bytes = 0
                    if graph:  # the step captured once, replayed: the GPU side without host overhead
                        cg = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(cg):
                            propagate_forward_reduced(x0u, x0i, rplan, K, red, fused=fused)
                        cg.replay()
                        torch.cuda.synchronize()
                        red.bytes = 0
                        t = time.perf_counter()
                        for _ in range(args.steps):
                            cg.replay()
                            red.bytes += moved_per_step
                        torch.cuda.synchronize()
                        del cg
                    else:
                        t = time.perf_counter()
                        for _ in range(args.steps):
                            propagate_forward_reduced(x0u, x0i, rplan, K, red, fused=fused)
                        host[order].append((time.perf_counter() - t) / args.steps * 1e3)
                        torch.cuda.synchronize()
                        moved_per_step = red.bytes / args.steps
                times[order].append((time.perf_counter() - t) / args.steps * 1e3)
                for dr in (rplan.users, rplan.partial):
                    dr.n_split_big = nb[id(dr)]
                moved = red.bytes / args.steps
            del rplan
        for order, ts in times.items():
            print(f"grid {R}x{F} reduce ({order}): rank compute {max(ts):.3f} ms/step (row groups "
                  f"{sorted({0, R - 1})}: {', '.join(f'{t:.3f}' for t in ts)}); ring all_reduce bytes per rank per "
                  f"step {moved / 1e6:.1f} MB" + (f"; host issue {max(host[order]):.3f} ms/step (no collectives)"
                                                   if host[order] else ""), flush=True)


if __name__ == "__main__":
    main()
