"""Probe: what bounds the C2 item pass? Same schedule and kernel, three column maps:
  real    the C2 plan as built;
  hot512  every neighbour id folded onto 512 rows per side (all gathers L1/L2-resident);
  seq     neighbour ids replaced by the row's own neighbour POSITION (streaming, no reuse).
python tools/gather_probe.py"""
import copy
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "movie-recommender-system-with-gnns_amd"))

import lgcn_amd  # noqa: E402
from lgcn_amd import synth  # noqa: E402
from lgcn_amd.plan import PropagationPlan  # noqa: E402


def main():
    dev = torch.device("cuda")
    g = synth.ml25m_shaped(seed=0)
    U, I, N = g.num_users, g.num_items, g.num_nodes
    ei = torch.from_numpy(g.edge_index).to(dev)
    K, d = 3, 64
    uw = torch.randn(U, d, device=dev) * 0.01
    iw = torch.randn(I, d, device=dev) * 0.01
    plan = PropagationPlan(ei, N, 256, side_split=U)
    col = plan.fwd.col.long()
    variants = {"real": plan.fwd.col}
    variants["hot512"] = torch.where(col < U, col % 512, U + (col - U) % 512).int()
    variants["hot64"] = torch.where(col < U, col % 64, U + (col - U) % 64).int()
    E = col.numel()
    variants["seq"] = (torch.arange(E, device=dev) % N).int()
    for rep in range(2):
        for name, c in variants.items():
            p = copy.copy(plan)
            p.fwd = copy.copy(plan.fwd)
            p.fwd.col = c.contiguous()
            times = []

            def timer(_d):
                class C:
                    def __enter__(s):
                        s.e0 = torch.cuda.Event(enable_timing=True)
                        s.e0.record()

                    def __exit__(s, *a):
                        e1 = torch.cuda.Event(enable_timing=True)
                        e1.record()
                        times.append((s.e0, e1))
                return C()

            with torch.no_grad():
                for _ in range(2):
                    lgcn_amd.propagate_forward(uw, iw, p, K)
                lgcn_amd.set_launch_timer(timer)
                for _ in range(10):
                    lgcn_amd.propagate_forward(uw, iw, p, K)
                torch.cuda.synchronize()
                lgcn_amd.set_launch_timer(None)
            ms = sorted(a.elapsed_time(b) for a, b in times)
            print(f"{name:8s} item pass median {ms[len(ms) // 2]:.3f} ms  min {ms[0]:.3f}", flush=True)


if __name__ == "__main__":
    main()
