"""A/B sweep of schedule parameters on the C2 graph, interleaved rounds in one process
(cdna_hip_programming.md §5.4 rule 24). Prints per-variant median/min ms per K=3 forward and
per item-pass launch."""
from __future__ import annotations

import argparse
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "movie-recommender-system-with-gnns_amd"))
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", default="64,128,256,512,1024")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--scale", type=float, default=1.0)
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
    plans = {c: PropagationPlan(ei, g.num_nodes, c) for c in map(int, args.chunks.split(","))}
    ref = None
    for c, p in plans.items():
        out = lgcn_amd.propagate_forward(uw, iw, p, K)
        if ref is None:
            ref = out
        rel = ((out - ref).abs().max() / ref.abs().max()).item()
        print(f"chunk {c}: items {p.fwd.n_items} splits {p.fwd.n_splits} partials {p.fwd.n_partials} "
              f"rel-diff vs first {rel:.2e}", file=sys.stderr)

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

    res = {c: {"step": [], "kernel": []} for c in plans}
    for _ in range(args.rounds):
        for c, p in plans.items():
            tm = Timer()
            lgcn_amd.set_launch_timer(tm)
            s0 = torch.cuda.Event(enable_timing=True)
            s1 = torch.cuda.Event(enable_timing=True)
            s0.record()
            for _ in range(args.reps):
                lgcn_amd.propagate_forward(uw, iw, p, K)
            s1.record()
            torch.cuda.synchronize()
            lgcn_amd.set_launch_timer(None)
            res[c]["step"].append(s0.elapsed_time(s1) / args.reps)
            res[c]["kernel"].append(sum(a.elapsed_time(b) for a, b in tm.pairs) / len(tm.pairs))
    out = {}
    for c, r in res.items():
        st, kn = sorted(r["step"]), sorted(r["kernel"])
        out[c] = {"step_ms_median": st[len(st) // 2], "step_ms_min": st[0], "kernel_ms_median": kn[len(kn) // 2],
                  "kernel_ms_min": kn[0], "edges_per_s": K * g.num_edges / (st[len(st) // 2] * 1e-3)}
        print(f"chunk {c}: step {out[c]['step_ms_median']:.3f} ms (min {st[0]:.3f}) kernel "
              f"{out[c]['kernel_ms_median']:.3f} ms  -> {out[c]['edges_per_s']:.3e} edges/s")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
