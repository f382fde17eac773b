"""CPU probe: the row-lazy Adam's replay work per C3 step (bench.py --workload train: ML-25M-shaped
graph, 90 % train split, 1024 parts, 32 parts per batch, one uniform negative item per user->item
edge). Walks the batch sequence for three epochs and prints, per step of the third, the rows the
step's Adam touches and how many zero-gradient steps each replays first (users / items).
python tools/adam_gap_probe.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "movie-recommender-system-with-gnns_amd"))

from lgcn_amd import cluster, synth  # noqa: E402


def main():
    t0 = time.time()
    g = synth.ml25m_shaped(seed=0)
    U, I, N = g.num_users, g.num_items, g.num_nodes
    tr = synth.train_split(g.edge_index, 0.9, seed=0)
    _, f, lists = cluster.cluster_batches(tr, N, 1024, 32)
    print(f"{len(lists)} batches, intra-part fraction {f:.3f}, mean {np.mean([b.shape[1] for b in lists]):.0f} "
          f"edges per batch ({time.time() - t0:.1f} s)")
    last = np.zeros(N, dtype=np.int64)
    rng = np.random.default_rng(0)
    nb = len(lists)
    for t in range(1, 3 * nb + 1):
        src, dst = lists[(t - 1) % nb]
        m = src < U
        negs = rng.integers(0, I, size=int(m.sum())) + U
        rows = np.unique(np.concatenate([src[m], dst[m], negs]))
        gap = (t - 1) - last[rows]
        if t > 2 * nb and t % 4 == 0:
            gu, gi = gap[rows < U], gap[rows >= U]
            print(f"step {t}: {rows.size} rows; users {gu.size} replaying {gu.sum()} steps (max {gu.max()}, "
                  f"mean {gu.mean():.1f}); items {gi.size} replaying {gi.sum()} (max {gi.max()}, mean {gi.mean():.1f})")
        last[rows] = t


if __name__ == "__main__":
    main()
