"""A/B the item-pass kernel variants (LGCN_SPMM_VARIANT) on the C2 graph: interleaved rounds in
one process, bitwise check against variant 0, per-launch and per-step medians."""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "movie-recommender-system-with-gnns_amd"))
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1,2,3,4,5,6")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--chunk", type=int, default=256)
    ap.add_argument("--side", type=int, default=-1, help="side_split (-1 = num_users)")
    ap.add_argument("--mixed", action="store_true", help="also time the unsided (global longest-first) schedule")
    args = ap.parse_args()

    import torch

    import lgcn_amd
    from lgcn_amd import synth
    from lgcn_amd.plan import PropagationPlan

    dev = torch.device("cuda:0")
    g = synth.ml25m_shaped(seed=0, scale=args.scale)
    ei = torch.from_numpy(g.edge_index).to(dev)
    d, K = args.dim, args.layers
    uw = torch.randn(g.num_users, d, device=dev) * 0.01
    iw = torch.randn(g.num_items, d, device=dev) * 0.01
    plans = {"sided": PropagationPlan(ei, g.num_nodes, args.chunk, g.num_users if args.side < 0 else args.side)}
    if args.mixed:
        plans["mixed"] = PropagationPlan(ei, g.num_nodes, args.chunk, 0)
    plan = plans["sided"]
    variants = [(int(v), p) for v in args.variants.split(",") for p in plans]
    os.environ["LGCN_SPMM_VARIANT"] = "0"
    ref = lgcn_amd.propagate_forward(uw, iw, plan, K)
    for v, pn in variants:
        os.environ["LGCN_SPMM_VARIANT"] = str(v)
        out = lgcn_amd.propagate_forward(uw, iw, plans[pn], K)
        print(f"variant {v}/{pn}: bitwise equal to variant 0: {bool(torch.equal(out, ref))}", file=sys.stderr)

    class Timer:
        def __init__(self):
            self.pairs = []

        def __call__(self, _d):
            t = self

            class C:
                def __enter__(s):
                    s.e0 = torch.cuda.Event(enable_timing=True)
                    s.e0.record()

                def __exit__(s, *a):
                    e1 = torch.cuda.Event(enable_timing=True)
                    e1.record()
                    t.pairs.append((s.e0, e1))

            return C()

    res = {v: {"step": [], "kernel": []} for v in variants}
    for _ in range(args.rounds):
        for v, pn in variants:
            os.environ["LGCN_SPMM_VARIANT"] = str(v)
            plan = plans[pn]
            tm = Timer()
            lgcn_amd.set_launch_timer(tm)
            s0 = torch.cuda.Event(enable_timing=True)
            s1 = torch.cuda.Event(enable_timing=True)
            s0.record()
            for _ in range(args.reps):
                lgcn_amd.propagate_forward(uw, iw, plan, K)
            s1.record()
            torch.cuda.synchronize()
            lgcn_amd.set_launch_timer(None)
            res[(v, pn)]["step"].append(s0.elapsed_time(s1) / args.reps)
            res[(v, pn)]["kernel"].append(sum(a.elapsed_time(b) for a, b in tm.pairs) / len(tm.pairs))
    out = {}
    for v, r in res.items():
        st, kn = sorted(r["step"]), sorted(r["kernel"])
        v = f"{v[0]}/{v[1]}"
        out[v] = {"step_ms": st[len(st) // 2], "kernel_ms": kn[len(kn) // 2], "kernel_ms_min": kn[0],
                  "edges_per_s": K * g.num_edges / (st[len(st) // 2] * 1e-3)}
        print(f"variant {v}: step {out[v]['step_ms']:.3f} ms  kernel {out[v]['kernel_ms']:.3f} ms "
              f"(min {kn[0]:.3f})  {out[v]['edges_per_s']:.3e} edges/s")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
