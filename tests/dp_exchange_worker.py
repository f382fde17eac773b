"""One rank of the data-parallel training check in tests/test_gpu_exchange.py (started as a
child process per rank; gloo over one GPU): trains the same Cluster-GCN batches several ways —
dense FusedAdam after an all_reduce of both gradients, the row-lazy Adam with the row-sparse
exchange, the owner-sharded exchange or the hybrid one (DP_VARIANTS hybrid / hybrid_graphs: items
all_reduced densely), and column-sharded (DP_VARIANTS cols / cols_graphs), each
eager and hipGraph-replayed — and saves the final tables and losses.

python tests/dp_exchange_worker.py RANK WORLD PORT OUT CLIP [BATCHES.npz]

With BATCHES.npz (U, I, b0, b1, ...: Cluster-GCN batch edge lists, e.g. C3's) the ranks train
those batches at d=128 (C4 rehearsal); otherwise a small subsampled graph at d=64."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "movie-recommender-system-with-gnns_amd"), ROOT, os.path.join(ROOT, "tests")]


class _Batch:
    def __init__(self, ei):
        self.edge_index = ei

    def to(self, device):
        return self


def main():
    rank, world, port, out, clip = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4], float(sys.argv[5])
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = port
    dist.init_process_group("gloo", rank=rank, world_size=world)
    gpu = torch.device("cuda:0")
    torch.cuda.set_device(gpu)

    import graphs
    from lgcn_amd import cluster as C
    from lgcn_amd import _ffi, tuning

    if os.environ.get("DP_DEVICE_COLLECTIVES") == "1":  # the RCCL branches, gloo carrying the bytes
        tuning.set_tuning(device_collectives=True)
    from lgcn_amd import distributed as D
    from lgcn_amd.optim import FusedAdam, RowLazyAdam
    from lgcn_amd.train_step import FusedTrainStep
    from models.light_gcn import LightGCN

    if len(sys.argv) > 6:
        import numpy as np

        z = np.load(sys.argv[6])
        U, I, d = int(z["U"]), int(z["I"]), 128
        lists = [z[k] for k in sorted((k for k in z.files if k.startswith("b")), key=lambda k: int(k[1:]))]
    else:
        U, I, ei = graphs.subsampled(U=2000, I=1000, pairs=8000, seed=4)
        part = C.partition_nodes(ei, U + I, 8)
        lists, d = C.intra_part_edges(ei, part, 8), 64
    batches = [_Batch(torch.from_numpy(x).to(gpu)) for x in lists]
    share = D.rank_share(len(batches), world, rank, seed=0, epoch=0)
    cap = D.exchange_capacity(batches, U)
    from lgcn_amd.owner import OwnerExchange, owner_capacity

    ocap = owner_capacity(batches, U, world, num_items=I)
    variants = os.environ.get("DP_VARIANTS", "dense,lazy,lazy_graphs,owner,owner_graphs").split(",")
    res = {}
    clip_ = None if clip == 0 else clip
    steps = int(os.environ.get("DP_STEPS", "12"))
    for name in variants:
        torch.manual_seed(0)
        cg = None
        if name.startswith("cols"):
            # column-sharded: every rank steps the same batches on its d / W columns
            from lgcn_amd.train_step import ColumnGroup

            cg = ColumnGroup(world, rank, d)
        m = LightGCN(U, I, num_layers=3, dim_h=d if cg is None else cg.d).to(gpu)
        ex = None
        if cg is not None:
            opt = RowLazyAdam(m.user_embedding.weight.data, m.item_embedding.weight.data, lr=1e-2,
                              max_grad_norm=clip_)
            step = FusedTrainStep(m, opt, lazy=True, cols=cg, graphs=name.endswith("_graphs"), neg_seed=7)
        elif name == "dense":
            opt = FusedAdam(m.parameters(), lr=1e-2, max_grad_norm=clip_, capturable=True)
            step = FusedTrainStep(m, opt, world=world, neg_seed=100 + rank)
        else:
            opt = RowLazyAdam(m.user_embedding.weight.data, m.item_embedding.weight.data, lr=1e-2,
                              max_grad_norm=clip_)
            if name.startswith("owner"):
                ex = OwnerExchange(ocap, U + I, d, gpu, world, rank, _ffi.load().lgcn_row_grad_norm_workspace_floats())
            elif name.startswith("hybrid"):
                ex = D.HybridExchange(D.user_exchange_capacity(batches, U), U, opt.gi, gpu, world)
            else:
                ex = D.RowExchange(cap, U + I, d, gpu, world)
            step = FusedTrainStep(m, opt, world=world, lazy=True, exchange=ex, graphs=name.endswith("_graphs"),
                                  neg_seed=100 + rank)  # per-rank negatives, the same for every variant
        losses = []
        for i in range(steps):
            order = share if cg is None else list(range(len(batches)))
            b = batches[order[i % len(order)]]
            if name.startswith("owner"):
                nxt = batches[share[(i + 1) % len(share)]] if i + 1 < steps else None
                losses.append(step.step(b, nxt).item())
            else:
                losses.append(step.step(b).item())
        step.sync()
        torch.cuda.synchronize()
        if name.startswith("owner"):
            ex.check_overflow()
        res[name] = {"losses": losses, "user": m.user_embedding.weight.detach().cpu(),
                     "item": m.item_embedding.weight.detach().cpu(),
                     "bytes_per_step": (ex.bytes / steps) if ex is not None and hasattr(ex, "bytes") else None}
    res["cap"] = cap
    res["ocap"] = ocap
    res["d"] = d
    torch.save(res, out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
