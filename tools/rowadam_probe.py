"""Probe: one C3-shaped row-Adam catch-up launch alone (lgcn_row_adam mode 0, d=128): the rows a
step's update replays (tools/adam_gap_probe.py) — 5,050 user rows 31 steps behind and 10,500 item
rows a few steps behind (geometric, mean ~4.5, at most 31) — on ML-25M-shaped tables. Times the
launch with HIP events (median of --reps; last[] and claim[] reset before each) and prints the
replayed row-steps. python tools/rowadam_probe.py [--reps 50]"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "movie-recommender-system-with-gnns_amd"))

from lgcn_amd.optim import RowLazyAdam  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--users", type=int, default=5050)
    ap.add_argument("--items", type=int, default=10500)
    ap.add_argument("--user-gap", type=int, default=31)
    args = ap.parse_args()
    dev = torch.device("cuda")
    U, I, d, T = 162_541, 59_047, 128, 64
    g = torch.Generator(device=dev).manual_seed(0)
    uw = torch.randn(U, d, device=dev, generator=g) * 0.1
    iw = torch.randn(I, d, device=dev, generator=g) * 0.1
    opt = RowLazyAdam(uw, iw, lr=1e-3, max_steps=1024)
    for t in (*opt.m, *opt.v):
        t.copy_(torch.rand(t.shape, device=dev, generator=g) * 1e-3)
    opt.step_dev.fill_(T)
    opt.steps = T
    rng = np.random.default_rng(0)
    users = rng.choice(U, args.users, replace=False)
    items = U + rng.choice(I, args.items, replace=False)
    rows = torch.from_numpy(np.concatenate([users, items]).astype(np.int32)).to(dev)
    gap_i = np.minimum(rng.geometric(1 / 4.5, args.items), 31)
    last0 = torch.full((U + I,), T, dtype=torch.int32, device=dev)
    last0[torch.from_numpy(users).to(dev)] = T - args.user_gap
    last0[torch.from_numpy(items).to(dev)] = torch.from_numpy((T - gap_i).astype(np.int32)).to(dev)
    replays = args.users * args.user_gap + int(gap_i.sum())
    ts = []
    for rep in range(args.reps + 3):
        opt.last.copy_(last0)
        opt.claim.fill_(-1)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        opt.catch_up(rows)
        b.record()
        torch.cuda.synchronize()
        if rep >= 3:
            ts.append(a.elapsed_time(b) * 1e3)
    print(f"row-Adam catch-up, d={d}: {args.users} users x {args.user_gap} + {args.items} items "
          f"(mean {gap_i.mean():.1f}) = {replays} row-replays: median {np.median(ts):.2f} us, min {min(ts):.2f} us",
          flush=True)


if __name__ == "__main__":
    main()
