"""Interleaved A/B of one lgcn_amd.tuning field on the C2 K-layer forward: bitwise check against
the first value, median/min ms per forward. (Round 5: the knobs are tuning fields, not environment
variables. A field read when a plan's schedule is built — slice_mb — needs a plan per value: one is
built for each.)
python tools/ab_tune.py --field spmm_index_rounds --values 0,2,8 [--dim 64]"""
from __future__ import annotations

import argparse
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "movie-recommender-system-with-gnns_amd"))
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--field", required=True)
    ap.add_argument("--values", default="0,1")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--layers", type=int, default=3)
    args = ap.parse_args()
    import torch

    import dataclasses

    import lgcn_amd
    from lgcn_amd import synth, tuning
    from lgcn_amd.plan import PropagationPlan

    ftype = {f.name: f.type for f in dataclasses.fields(tuning.Tuning)}[args.field]

    def cast(v):
        if "bool" in str(ftype):
            return v not in ("0", "false", "False")
        if "float" in str(ftype):
            return None if v == "None" else float(v)
        if "int" in str(ftype):
            return int(v)
        return v

    dev = torch.device("cuda:0")
    g = synth.ml25m_shaped(seed=0)
    ei = torch.from_numpy(g.edge_index).to(dev)
    d, K = args.dim, args.layers
    uw = torch.randn(g.num_users, d, device=dev) * 0.01
    iw = torch.randn(g.num_items, d, device=dev) * 0.01
    vals = args.values.split(",")
    plans, outs = {}, {}
    for v in vals:
        tuning.set_tuning(**{args.field: cast(v)})
        plans[v] = PropagationPlan(ei, g.num_nodes, side_split=g.num_users)
        outs[v] = lgcn_amd.propagate_forward(uw, iw, plans[v], K)
        print(f"{args.field}={v}: bitwise equal to {vals[0]}: {bool(torch.equal(outs[v], outs[vals[0]]))}", flush=True)
    res = {v: [] for v in vals}
    for _ in range(args.rounds):
        for v in vals:
            tuning.set_tuning(**{args.field: cast(v)})
            plan = plans[v]
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.reps):
                lgcn_amd.propagate_forward(uw, iw, plan, K)
            b.record()
            torch.cuda.synchronize()
            res[v].append(a.elapsed_time(b) / args.reps)
    for v in vals:
        t = sorted(res[v])
        print(f"{args.field}={v}: median {t[len(t) // 2]:.3f} ms  min {t[0]:.3f} ms  "
              f"{K * g.num_edges / (t[len(t) // 2] * 1e-3):.3e} edges/s", flush=True)


if __name__ == "__main__":
    main()
