"""Where does a Cluster-GCN training step spend its time? Host-side phase timings (no syncs
inside the step) + wall per step, for torch Adam vs FusedAdam vs torch fused Adam, on the C3
setup at a reduced number of parts."""
from __future__ import annotations

import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "movie-recommender-system-with-gnns_amd"))
sys.path.insert(0, str(ROOT))


def main():
    import numpy as np
    import torch

    from data.dataset_handler import Data
    from lgcn_amd import cluster, synth
    from lgcn_amd.optim import FusedAdam
    from models.light_gcn import LightGCN
    from utils.train_test import bpr_loss, compute_embeddings

    dev = torch.device("cuda:0")
    g = synth.ml25m_shaped(seed=0, scale=1.0)
    N = g.num_nodes
    rng = np.random.default_rng(0)
    perm = rng.permutation(g.num_edges)
    train_ei = np.ascontiguousarray(g.edge_index[:, np.sort(perm[: int(0.9 * g.num_edges)])])
    part = cluster.partition_nodes(train_ei, N, 1024)
    lists = cluster.intra_part_edges(train_ei, part, 1024)
    batches = [Data(edge_index=torch.from_numpy(np.concatenate(lists[b:b + 32], axis=1)).to(dev), num_nodes=N)
               for b in range(0, 1024, 32)]
    for name in ("torch", "fused", "torch_fused"):
        torch.manual_seed(0)
        model = LightGCN(g.num_users, g.num_items, num_layers=3, dim_h=128).to(dev)
        if name == "torch":
            opt = torch.optim.Adam(model.parameters(), lr=1e-3)
        elif name == "fused":
            opt = FusedAdam(model.parameters(), lr=1e-3, max_grad_norm=1)
        else:
            opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True)
        params = list(model.parameters())
        phases = {"fwd": 0.0, "loss": 0.0, "bwd": 0.0, "opt": 0.0}
        for b in batches:  # warm: plans
            opt.zero_grad()
            bpr_loss(*compute_embeddings(model, b, dev)).backward()
            if name != "fused":
                torch.nn.utils.clip_grad_norm_(params, 1)
            opt.step()
        torch.cuda.synchronize()
        steps = 64
        t_all = time.perf_counter()
        for i in range(steps):
            b = batches[i % len(batches)]
            t0 = time.perf_counter()
            opt.zero_grad()
            embs = compute_embeddings(model, b, dev)
            t1 = time.perf_counter()
            loss = bpr_loss(*embs)
            t2 = time.perf_counter()
            loss.backward()
            t3 = time.perf_counter()
            if name != "fused":
                torch.nn.utils.clip_grad_norm_(params, 1)
            opt.step()
            t4 = time.perf_counter()
            phases["fwd"] += t1 - t0
            phases["loss"] += t2 - t1
            phases["bwd"] += t3 - t2
            phases["opt"] += t4 - t3
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t_all) / steps * 1e3
        print(f"{name:12s} wall {wall:.3f} ms/step  host: " +
              "  ".join(f"{k} {v / steps * 1e3:.3f}" for k, v in phases.items()), flush=True)


if __name__ == "__main__":
    main()
