"""Probe: per-table slice counts of the source-sliced C2 forward. The user table (gathered by
item rows) and the item table (gathered by user rows) are cut into ku and ki slices independently
(lgcn_amd.sliced.slice_bounds cuts both to one byte size). Times the K-layer forward per
(ku, ki, chunk) and checks it against the default schedule (max row-relative difference).
python tools/slice_split_probe.py [--cfg 5x2,10x2,...] [--chunks 256,512]"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "movie-recommender-system-with-gnns_amd"))

import lgcn_amd  # noqa: E402
from lgcn_amd import synth  # noqa: E402
from lgcn_amd.plan import PropagationPlan  # noqa: E402
from lgcn_amd.sliced import build_sliced, propagate_forward_sliced  # noqa: E402


def bounds_for(N, U, ku, ki):
    I = N - U
    return sorted(set([0] + [(U * i) // ku for i in range(1, ku + 1)] + [U + (I * i) // ki for i in range(1, ki + 1)]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="5x2,8x2,10x2,12x2,16x2,5x3,10x3,10x4")
    ap.add_argument("--chunks", default="256")
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda")
    g = synth.ml25m_shaped(seed=0)
    U, I, N, E = g.num_users, g.num_items, g.num_nodes, g.num_edges
    ei = torch.from_numpy(g.edge_index).to(dev)
    K, d = args.layers, args.dim
    gen = torch.Generator(device=dev).manual_seed(0)
    uw = torch.randn(U, d, device=dev, generator=gen) * 0.01
    iw = torch.randn(I, d, device=dev, generator=gen) * 0.01

    def bench(fn):
        with torch.no_grad():
            for _ in range(3):
                out = fn()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(args.steps):
                out = fn()
            torch.cuda.synchronize()
        return out, (time.perf_counter() - t) / args.steps * 1e3

    plan = PropagationPlan(ei, N, 256, side_split=U)
    runs = {"default": (None, lambda: lgcn_amd.propagate_forward(uw, iw, plan, K))}
    ref = runs["default"][1]()
    for chunk in [int(c) for c in args.chunks.split(",")]:
        for cfg in args.cfg.split(","):
            ku, ki = (int(v) for v in cfg.split("x"))
            sd = build_sliced(plan.fwd, N, bounds_for(N, U, ku, ki), chunk)
            runs[f"ku={ku:2d} ki={ki:2d} chunk={chunk:4d}"] = (sd, lambda s=sd: propagate_forward_sliced(uw, iw, s, K))
    # interleaved rounds: every configuration timed once per round, medians reported
    times = {n: [] for n in runs}
    for _ in range(args.rounds):
        for n, (_, fn) in runs.items():
            times[n].append(bench(fn)[1])
    for n, (sd, fn) in runs.items():
        out = fn()
        rel = ((out - ref).abs().max(1).values / ref.abs().max(1).values.clamp_min(1e-30)).max().item()
        t = sorted(times[n])
        ms = t[len(t) // 2]
        desc = f"{sd.n_launches:2d} launches, {sd.n_splits:5d} hub rows, " if sd is not None else ""
        print(f"{n}: {desc}{ms:.3f} ms/step  {K * E / ms / 1e6:.2f} e9 edges/s  max row-rel diff {rel:.2e}",
              flush=True)


if __name__ == "__main__":
    main()
