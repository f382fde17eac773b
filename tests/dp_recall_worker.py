"""One rank of the data-parallel Recall check in tests/test_gpu_dp_recall.py (one child process
per rank, gloo over one GPU; W = 1 runs the same code with one rank).

C1-sized graph (BASELINE configs[0]: U = 1000, I = 600, 25k pairs -> E = 50k, K = 2, d = 64),
its 90/5/5 split, PARTS Cluster-GCN parts, one part per step per rank (the reference's
batch_size = 1), the default fused step with the row-lazy Adam(1e-3) + clip 1 and, at W > 1,
the row-sparse gradient exchange (lgcn_amd.distributed.RowExchange). After EPOCHS epochs rank 0
scores Recall@20 / @100 on the validation edges through the reference harness
(utils/train_test.py compute_embeddings + compute_recall_at_k, numpy seed 5) and saves them.

python tests/dp_recall_worker.py RANK WORLD PORT OUT EPOCHS PARTS"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "movie-recommender-system-with-gnns_amd"), ROOT, os.path.join(ROOT, "tests")]


class _Batch:
    def __init__(self, ei):
        self.edge_index = ei

    def to(self, device):
        return _Batch(self.edge_index.to(device))


def c1_split(parts: int):
    """(U, I, Cluster-GCN part edge lists, validation edge_index): the C1 graph of
    test_recall_parity_c1_size."""
    import numpy as np

    from lgcn_amd import cluster, synth

    g = synth.bipartite(1000, 600, 25_000, seed=11)
    E = g.num_edges
    perm = np.random.default_rng(0).permutation(E)
    n_tr, n_va = int(0.9 * E), int(0.05 * E)
    train = np.ascontiguousarray(g.edge_index[:, np.sort(perm[:n_tr])])
    val = np.ascontiguousarray(g.edge_index[:, np.sort(perm[n_tr:n_tr + n_va])])
    _, _, lists = cluster.cluster_batches(train, g.num_nodes, parts, 1)
    return g.num_users, g.num_items, [p for p in lists if p.shape[1]], val


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    epochs, parts = int(sys.argv[5]), int(sys.argv[6])
    import numpy as np
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = port
    dist.init_process_group("gloo", rank=rank, world_size=world)
    gpu = torch.device("cuda:0")
    torch.cuda.set_device(gpu)

    from lgcn_amd import distributed as D
    from lgcn_amd.optim import RowLazyAdam
    from lgcn_amd.train_step import FusedTrainStep
    from models.light_gcn import LightGCN
    from oracle.lgconv_torch import OracleLightGCN
    from utils import train_test as TT

    U, I, lists, val = c1_split(parts)
    batches = [_Batch(torch.from_numpy(x).to(gpu)) for x in lists]
    torch.manual_seed(0)
    ref_init = OracleLightGCN(U, I, num_layers=2, dim_h=64)  # the reference's seed-0 init
    m = LightGCN(U, I, num_layers=2, dim_h=64).to(gpu)
    m.load_state_dict(ref_init.state_dict())
    opt = RowLazyAdam(m.user_embedding.weight.data, m.item_embedding.weight.data, lr=1e-3, max_grad_norm=1.0)
    ex = D.RowExchange(D.exchange_capacity(batches, U), U + I, 64, gpu, world) if world > 1 else None
    step = FusedTrainStep(m, opt, world=world, lazy=True, exchange=ex)
    steps = 0
    for epoch in range(epochs):
        for i, b in enumerate(D.rank_share(len(batches), world, rank, seed=0, epoch=epoch)):
            torch.cuda.manual_seed(100_000 * epoch + 100 * i + rank)  # per-rank negatives
            step.step(batches[b])
            steps += 1
        step.sync()
    torch.cuda.synchronize()
    if rank == 0:
        with torch.no_grad():
            embs = TT.compute_embeddings(m, _Batch(torch.from_numpy(val)).to(gpu), gpu)
            rec = {}
            for k in (20, 100):
                np.random.seed(5)
                rec[k] = TT.compute_recall_at_k((embs[1], embs[3], embs[5]), k=k)
        with open(out, "w") as f:
            json.dump({"world": world, "steps_per_rank": steps, "parts": len(batches), "recall": rec}, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
