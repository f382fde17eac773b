"""Probe: LDS-staged hot sources (lgcn_spmm_hot) vs the source-sliced item pass on the C2 graph.
python tools/hot_probe.py [--hot 0,128,256,384] [--block 256,512,1024] [--dim 64]
Checks one layer bitwise against the sliced path, then times K-layer forwards interleaved."""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "movie-recommender-system-with-gnns_amd"))

import lgcn_amd  # noqa: E402
from lgcn_amd import _ffi, synth  # noqa: E402
from lgcn_amd.plan import PropagationPlan  # noqa: E402
from lgcn_amd.sliced import SlicedDirection, attach_hot, spmm_sliced  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hot", default="128,256,384")
    ap.add_argument("--block", default="512,1024")
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--layers", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda")
    g = synth.ml25m_shaped(seed=0)
    U, I, N, E = g.num_users, g.num_items, g.num_nodes, g.num_edges
    ei = torch.from_numpy(g.edge_index).to(dev)
    K, d = args.layers, args.dim
    gen = torch.Generator(device=dev).manual_seed(0)
    uw = torch.randn(U, d, device=dev, generator=gen) * 0.01
    iw = torch.randn(I, d, device=dev, generator=gen) * 0.01
    plan = PropagationPlan(ei, N, 256, side_split=U)
    sd = plan.schedule("fwd", d)
    assert isinstance(sd, SlicedDirection), "C2 should take the sliced schedule"
    s = _ffi.stream_of(dev)
    run = torch.empty((N, d), device=dev)
    part = torch.empty((max(sd.n_partials, 1), d), device=dev)

    def one_layer():
        o = torch.empty((N, d), device=dev)
        spmm_sliced(sd, N, d, (uw, iw, U), None, (o, None, N), None, _ffi.EPI_STORE, 1.0, 1.0, run, part, s)
        return o

    def bench(fn):
        with torch.no_grad():
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(args.steps):
                fn()
            torch.cuda.synchronize()
        return (time.perf_counter() - t) / args.steps * 1e3

    sd.hot = None
    ref1 = one_layer()
    ref = lgcn_amd.propagate_forward(uw, iw, plan, K)
    variants = [(0, 0)] + [(h, b) for h in map(int, args.hot.split(",")) for b in map(int, args.block.split(","))]
    for h, b in variants:
        attach_hot(sd, N, d, h, b)
        o1 = one_layer()
        out = lgcn_amd.propagate_forward(uw, iw, plan, K)
        torch.cuda.synchronize()
        eq1, eq = torch.equal(o1, ref1), torch.equal(out, ref)
        grid = sd.hot.grid[0] if sd.hot else 0
        print(f"hot={h:4d} block={b:4d} grid={grid:5d}: one layer bitwise {eq1}, K={K} forward bitwise {eq}",
              flush=True)
    times = {v: [] for v in variants}
    for rep in range(3):
        for h, b in variants:
            attach_hot(sd, N, d, h, b)
            times[(h, b)].append(bench(lambda: lgcn_amd.propagate_forward(uw, iw, plan, K)))
    for (h, b), ts in times.items():
        ms = min(ts)
        print(f"hot={h:4d} block={b:4d}: {ms:.3f} ms/step  {K * E / ms / 1e6:.2f} e9 edges/s  (reps {ts})",
              flush=True)


if __name__ == "__main__":
    main()
