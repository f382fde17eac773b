"""One rank of the data-parallel Recall check in tests/test_gpu_dp_recall.py (one child process
per rank, gloo over one GPU; W = 1 runs the same code with one rank).

C1-sized graph (BASELINE configs[0]: U = 1000, I = 600, 25k pairs -> E = 50k, K = 2, d = 64),
its 90/5/5 split, PARTS Cluster-GCN parts, one part per step per rank (the reference's
batch_size = 1), the default fused step with the row-lazy Adam(1e-3) + clip 1 and, at W > 1,
the row-sparse gradient exchange (lgcn_amd.distributed.RowExchange). After EPOCHS epochs rank 0
scores Recall@20 / @100 on the validation edges through the reference harness
(utils/train_test.py compute_embeddings + compute_recall_at_k, numpy seed 5) and saves them.

MODE "cols" (column-sharded training, lgcn_amd.train_step.ColumnGroup): every rank trains the
reference's schedule — every part, one per step, the same negatives — on its d / W columns; the
tables are gathered to rank 0 for Recall. MODE "plain": the same schedule and negatives without
the column split (W = 1).

LR_SCALE (dp only, default 1): the data-parallel Adam's lr is 1e-3 * LR_SCALE (tools/dp_lr_probe.py).

MODE "hybrid": data parallel with lgcn_amd.distributed.HybridExchange (items all_reduced densely).

python tests/dp_recall_worker.py RANK WORLD PORT OUT EPOCHS PARTS [MODE: dp | hybrid | cols | plain] [LR_SCALE]"""
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


def gather_columns(m, cg, world):
    """The full-width (user, item) tables on rank 0 from every rank's columns (CPU tensors)."""
    import torch
    import torch.distributed as dist

    u, i = m.user_embedding.weight.detach(), m.item_embedding.weight.detach()
    if cg is None or world == 1:
        return u.cpu().clone(), i.cpu().clone()
    us = [torch.empty_like(u) for _ in range(world)]
    its = [torch.empty_like(i) for _ in range(world)]
    dist.all_gather(us, u.contiguous())
    dist.all_gather(its, i.contiguous())
    return torch.cat([x.cpu() for x in us], 1), torch.cat([x.cpu() for x in its], 1)


def gather_tensor_columns(t, cg, world):
    """[n, d] on rank 0 from every rank's [n, d / W] columns (CPU)."""
    import torch
    import torch.distributed as dist

    if cg is None or world == 1:
        return t.cpu().clone()
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t.contiguous())
    return torch.cat([x.cpu() for x in parts], 1)


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    epochs, parts = int(sys.argv[5]), int(sys.argv[6])
    mode = sys.argv[7] if len(sys.argv) > 7 else "dp"
    lr_scale = float(sys.argv[8]) if len(sys.argv) > 8 and mode in ("dp", "hybrid") else 1.0
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

    from lgcn_amd.train_step import ColumnGroup

    U, I, lists, val = c1_split(parts)
    batches = [_Batch(torch.from_numpy(x).to(gpu)) for x in lists]
    torch.manual_seed(0)
    ref_init = OracleLightGCN(U, I, num_layers=2, dim_h=64)  # the reference's seed-0 init
    cg = ColumnGroup(world, rank, 64) if mode == "cols" else None
    c0, c1 = cg.cols if cg is not None else (0, 64)
    m = LightGCN(U, I, num_layers=2, dim_h=c1 - c0).to(gpu)
    with torch.no_grad():
        m.user_embedding.weight.copy_(ref_init.user_embedding.weight[:, c0:c1])
        m.item_embedding.weight.copy_(ref_init.item_embedding.weight[:, c0:c1])
    opt = RowLazyAdam(m.user_embedding.weight.data, m.item_embedding.weight.data, lr=1e-3 * lr_scale,
                      max_grad_norm=1.0)
    if mode == "dp":
        ex = D.RowExchange(D.exchange_capacity(batches, U), U + I, 64, gpu, world) if world > 1 else None
        step = FusedTrainStep(m, opt, world=world, lazy=True, exchange=ex, neg_seed=1000 + rank)
    elif mode == "hybrid":  # data parallel, the item gradient table all_reduced densely
        ex = D.HybridExchange(D.user_exchange_capacity(batches, U), U, opt.gi, gpu, world)
        step = FusedTrainStep(m, opt, world=world, lazy=True, exchange=ex, neg_seed=1000 + rank)
    else:  # the reference's schedule on every rank, the same negatives everywhere
        step = FusedTrainStep(m, opt, lazy=True, cols=cg, neg_seed=7)
    steps, losses, first_tables, first_grads = 0, [], None, None
    for epoch in range(epochs):
        sched_world, sched_rank = (world, rank) if mode in ("dp", "hybrid") else (1, 0)
        for i, b in enumerate(D.rank_share(len(batches), sched_world, sched_rank, seed=0, epoch=epoch)):
            losses.append(float(step.step(batches[b]).item()))
            steps += 1
            if steps == 1 and mode not in ("dp", "hybrid"):
                step.sync()
                first_tables = gather_columns(m, cg, world)
                # the first step's gradient rows (touched rows + first-occurrence negatives outside them)
                st = step.state(batches[b].edge_index)
                negs = st.neg[st.c2flag.bool()] + U
                negs = negs[st.plan.touched[negs] == 0]
                ids = torch.cat([st.touched_rows.long(), negs]).sort().values
                g = torch.cat([opt.gu, opt.gi])[ids]
                first_grads = (ids.cpu(), gather_tensor_columns(g, cg, world))
        step.sync()
    torch.cuda.synchronize()
    full = gather_columns(m, cg, world) if mode not in ("dp", "hybrid") else None
    if rank == 0 and mode not in ("dp", "hybrid"):
        torch.save({"losses": losses, "first": first_tables, "first_grads": first_grads, "final": full}, out + ".pt")
    if rank == 0:
        if full is not None:  # score the gathered full-width tables
            m = LightGCN(U, I, num_layers=2, dim_h=64).to(gpu)
            with torch.no_grad():
                m.user_embedding.weight.copy_(full[0])
                m.item_embedding.weight.copy_(full[1])
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
