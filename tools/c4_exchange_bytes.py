"""Bytes each rank receives per C4 training step (C3 batches: the ML-25M-shaped graph, 1024 parts,
32 per batch, d = 128) for the replicated row exchange (lgcn_amd.distributed.RowExchange: one
all_gather of every rank's record block) and the owner-sharded one (lgcn_amd.owner.OwnerExchange:
two all_to_alls of per-destination blocks + the clip norm's partials), at W = 2, 4, 8, from the
capacities each would allocate; plus the owner mode's once-per-epoch all_gather of the owned rows
(sync()) spread over the epoch's steps. Host only. python tools/c4_exchange_bytes.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "movie-recommender-system-with-gnns_amd"))

from lgcn_amd import cluster, synth  # noqa: E402
from lgcn_amd import distributed as D  # noqa: E402
from lgcn_amd.owner import owner_capacity  # noqa: E402


class _B:
    def __init__(self, ei):
        self.edge_index = ei


def main():
    d, norm_parts = 128, 2048
    g = synth.ml25m_shaped(seed=0)
    train = synth.train_split(g.edge_index, 0.9, seed=0)
    _, f_intra, lists = cluster.cluster_batches(train, g.num_nodes, 1024, 32)
    batches = [_B(torch.from_numpy(x)) for x in lists]
    U, I, N = g.num_users, g.num_items, g.num_nodes
    cap = D.exchange_capacity(batches, U)
    cap += cap % 2
    rep_blk = cap * (d + 2) * 4
    print(f"C3 batches: {len(batches)}, f_intra {f_intra:.4f}, replicated slots per rank {cap} "
          f"({rep_blk / 1e6:.2f} MB record block)")
    for W in (2, 4, 8):
        ocap = owner_capacity(batches, U, W, num_items=I)
        blk = ocap * (d + 2) + 2 * ocap
        blk += (-blk) % 4
        steps_per_epoch = len(batches) // W
        per = (N + W - 1) // W
        step_bytes = (W - 1) * (blk * 4 + ocap * d * 4 + norm_parts * 4)
        sync_bytes = (W - 1) * per * d * 4 / steps_per_epoch
        rep = (W - 1) * rep_blk
        print(f"W={W}: replicated {rep / 1e6:.1f} MB/step | owner {step_bytes / 1e6:.1f} MB/step "
              f"(+ {sync_bytes / 1e6:.1f} MB/step of the per-epoch sync at {steps_per_epoch} steps/epoch) "
              f"[owner cap {ocap} slots per destination]")


if __name__ == "__main__":
    main()
