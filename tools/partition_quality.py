"""Partition quality (fraction of edges kept intra-part) of the host partitioner
(lgcn_partition_edges) on a planted-community bipartite graph with a known ground truth and on
the ML-25M-shaped synthetic graph. CPU only. python tools/partition_quality.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "movie-recommender-system-with-gnns_amd"))
from lgcn_amd import cluster, synth  # noqa: E402


def main():
    g, truth = synth.planted_bipartite(40000, 16000, 256)
    N, ei = g.num_nodes, g.edge_index
    print(f"planted: N={N} E={ei.shape[1]} k=256 ground truth intra={cluster.intra_fraction(ei, truth):.4f}")
    for passes in (1, 4, 8):
        t = time.time()
        p = cluster.partition_nodes(ei, N, 256, passes=passes)
        print(f"  passes={passes}: intra={cluster.intra_fraction(ei, p):.4f} ({time.time() - t:.2f} s)")
    for scale, k in ((0.05, 64), (1.0, 1024)):
        g = synth.ml25m_shaped(seed=0, scale=scale)
        t = time.time()
        p = cluster.partition_nodes(g.edge_index, g.num_nodes, k)
        print(f"ml25m-shaped scale={scale} k={k}: intra={cluster.intra_fraction(g.edge_index, p):.4f} "
              f"(random {1 / k:.4f}) ({time.time() - t:.1f} s)")
    # C3 scale with a known answer: the ML-25M-sized planted-community graph, its 90 % train
    # split, 1024 parts, 32-part batches (what bench.py --workload train --graph planted runs)
    g, truth = synth.planted_ml25m(1024)
    train = synth.train_split(g.edge_index, 0.9, seed=0)
    t = time.time()
    p, f, batches = cluster.cluster_batches(train, g.num_nodes, 1024, 32)
    eb = np.array([b.shape[1] for b in batches])
    sz = np.bincount(p, minlength=1024)
    print(f"planted ML-25M-sized (U={g.num_users} I={g.num_items} E={g.num_edges}, 1024 communities): "
          f"train intra: partitioner {f:.4f} vs ground truth {cluster.intra_fraction(train, truth):.4f} "
          f"({f / cluster.intra_fraction(train, truth):.3f} of truth; random {1 / 1024:.4f}); part sizes "
          f"{sz.min()}-{sz.max()}; 32-part batches: mean {eb.mean():.0f} edges (min {eb.min()}, max {eb.max()}) "
          f"({time.time() - t:.1f} s)")


if __name__ == "__main__":
    main()
