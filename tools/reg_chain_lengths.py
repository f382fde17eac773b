"""the longest sequential reg-sum chain (n copies of kreg * W[r] added in order,
csrc/lgcn_bpr.hip reg_sum) a planted-graph batch gives one lane group: the largest number of
(user, positive) keys on one row of a batch (k_reg_rows) and the largest number of a step's B
uniform negatives on one item (lgcn_grouped_reg_add). Host only. python tools/reg_chain_lengths.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "movie-recommender-system-with-gnns_amd"))

from lgcn_amd import cluster, synth  # noqa: E402


def main():
    g, _ = synth.planted_ml25m(1024)
    U, I, N = g.num_users, g.num_items, g.num_nodes
    train = synth.train_split(g.edge_index, 0.9, seed=0)
    _, f_intra, lists = cluster.cluster_batches(train, N, 1024, 32)
    rng = np.random.default_rng(0)
    worst_fixed, worst_neg, Bs = 0, 0, []
    for ei in lists:
        src, dst = ei
        users = src[src < U]
        pos = dst[dst >= U]
        B = users.size
        Bs.append(B)
        keys = np.concatenate([users, pos])  # one (user, positive) key per row occurrence
        worst_fixed = max(worst_fixed, int(np.bincount(keys, minlength=N).max()))
        worst_neg = max(worst_neg, int(np.bincount(rng.integers(0, I, B), minlength=I).max()))
    print(f"planted batches: {len(lists)}, f_intra {f_intra:.4f}, B {min(Bs)}..{max(Bs)}; longest reg chain: "
          f"fixed rows {worst_fixed} keys on one row, negatives {worst_neg} draws on one item")


if __name__ == "__main__":
    main()
