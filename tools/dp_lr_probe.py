"""Data-parallel Recall against the reference harness as a function of the DP Adam's lr scale
(W ranks average W parts' gradients per step, so an epoch is W-times fewer steps): runs
tests/test_gpu_dp_recall.py's C1 setup at W ranks (gloo on one GPU) for each scale and prints
|dRecall@20| and |dRecall@100|. python tools/dp_lr_probe.py [--world 8] [--scales 1,2,4,8] [--epochs 5]"""
import argparse
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "movie-recommender-system-with-gnns_amd"), ROOT]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--scales", default="1,2,4,8")
    ap.add_argument("--epochs", type=int, default=5)
    args = ap.parse_args()
    import test_gpu_dp_recall as T

    ref = T._reference_harness(args.epochs)
    print(f"reference harness, {args.epochs} epochs: Recall@20 {ref['20']:.5f} Recall@100 {ref['100']:.5f}", flush=True)
    tmp = tempfile.mkdtemp()
    for s in (float(x) for x in args.scales.split(",")):
        r = T._run_ranks(args.world, os.path.join(tmp, f"dp_{s}.json"), "dp", lr_scale=s, epochs=args.epochs)
        d20, d100 = r["recall"]["20"] - ref["20"], r["recall"]["100"] - ref["100"]
        print(f"W={args.world} lr x{s:g}: Recall@20 {r['recall']['20']:.5f} (d {d20:+.5f}) Recall@100 "
              f"{r['recall']['100']:.5f} (d {d100:+.5f})", flush=True)


if __name__ == "__main__":
    main()
