"""Headline benchmark: edges propagated/s of K-layer LightGCN propagation (BASELINE.json metric).

Workload (BASELINE.json configs[1]): MovieLens-25M-shaped full bipartite graph
(U=162,541, I=59,047, 12.45M unique rating>=4 pairs -> E = 24.9M directed edges), K=3, d=64,
fp32. One step = one full K-layer forward propagation (LightGCN.forward semantics, reference
models/light_gcn.py:28-40) with the plan (CSR + gcn_norm + schedule) already built and the
embedding tables resident in HBM. value = K * E * (graphs processed) / wall time.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): one process per
GPU. C2 is replicas only (the full-graph SpMM does not split without a per-layer
exchange): each rank propagates its own independent graph instance (seed = rank), no data-path
collective (scaling: weak). C5 (--config c5) is feature-sharded: one graph, d/N columns per
rank, no collective (scaling: strong). The barrier and the max-over-ranks time go over RCCL.

Also reported (one JSON line on rank 0):
  roofline     — achieved algorithmic GB/s of the dominant kernel (the item pass, k_spmm_vec;
                 at C2 one launch per source slice, lgcn_amd.sliced), timed live with HIP events
                 on its launching stream, vs the 8 TB/s HBM peak; bytes per layer =
                 E*(4d+8) + N*(4d+8), per launch = that / launches per layer.
  cpu_baseline — the reference's CPU op sequence (PyG 2.4.0 LGConv restated with torch CPU
                 primitives, oracle/lgconv_torch.py) on a bounded sample, rank 0, N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "movie-recommender-system-with-gnns_amd"))
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class LaunchTimer:
    """HIP-event brackets around each dominant-kernel launch, on the launching stream."""

    def __init__(self):
        import torch

        self.torch = torch
        self.pairs = []
        self.active = False

    def __call__(self, d):
        timer = self

        class _Ctx:
            def __enter__(self_):
                if timer.active:
                    s = timer.torch.cuda.Event(enable_timing=True)
                    s.record(timer.torch.cuda.current_stream())
                    self_.s = s

            def __exit__(self_, *exc):
                if timer.active:
                    e = timer.torch.cuda.Event(enable_timing=True)
                    e.record(timer.torch.cuda.current_stream())
                    timer.pairs.append((self_.s, e))
                return False

        return _Ctx()

    def mean_ms(self):
        if not self.pairs:
            return None
        return sum(s.elapsed_time(e) for s, e in self.pairs) / len(self.pairs)


def load_traffic(workload: str):
    """HBM bytes per launch of the dominant kernel from a committed PMC profile (or None)."""
    p = ROOT / "profiles" / "pmc_traffic.json"
    if not p.exists():
        return None
    try:
        data = json.loads(p.read_text())
        ent = data.get(workload)
        return None if ent is None else ent.get("hbm_bytes_per_launch")
    except Exception:
        return None


def kernel_lpr(d):
    """Template of the item-pass instance lgcn_spmm launches for width d (csrc/lgcn_spmm.hip)."""
    return {4: "1,1,8", 8: "2,1,8", 16: "4,1,8", 32: "8,1,8", 64: "16,1,8", 128: "32,1,8", 256: "64,1,8",
            512: "64,2,4", 1024: "64,4,2"}.get(d, "scalar")


def init_dist(backend, dev):
    import torch.distributed as dist

    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group(backend)


def cpu_baseline(graph, K, d, seconds_budget=20.0):
    """Reference CPU path (torch primitives of PyG 2.4.0 LGConv) on a bounded edge sample."""
    import numpy as np
    import torch

    from oracle.lgconv_torch import time_csr_forward, time_reference_forward

    threads = min(16, len(os.sched_getaffinity(0)))
    torch.set_num_threads(threads)
    E = graph.num_edges
    frac = 0.1 if E > 5_000_000 else 1.0
    rng = np.random.default_rng(0)
    keep = np.sort(rng.choice(E, int(E * frac), replace=False)) if frac < 1 else np.arange(E)
    ei = torch.from_numpy(np.ascontiguousarray(graph.edge_index[:, keep]))
    g = torch.Generator().manual_seed(0)
    uw = torch.randn(graph.num_users, d, generator=g) * 0.01
    iw = torch.randn(graph.num_items, d, generator=g) * 0.01
    t0 = time.perf_counter()
    t = time_reference_forward(uw, iw, ei, K, reps=1)
    reps = max(1, min(5, int(seconds_budget / max(t, 1e-3)) - 1))
    if reps > 1:
        t = time_reference_forward(uw, iw, ei, K, reps=reps)
    log(f"cpu_baseline: {ei.shape[1]} edges, {threads} threads, {t:.3f} s/forward "
        f"({time.perf_counter() - t0:.1f} s total)")
    # second CPU baseline: the whole C2 graph as one CSR matrix, torch.sparse.mm per layer
    full = torch.from_numpy(graph.edge_index)
    t1 = time.perf_counter()
    tc = time_csr_forward(uw, iw, full, K, reps=3)
    log(f"cpu_baseline csr: {full.shape[1]} edges, {tc:.3f} s/forward ({time.perf_counter() - t1:.1f} s total)")
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            model = next(line.split(":", 1)[1].strip() for line in f if line.startswith("model name"))
    except (OSError, StopIteration):
        pass
    return {"value": K * ei.shape[1] / t, "unit": "edges/s", "cores": threads, "kind": "port", "cpu_model": model,
            "csr_spmm": {"value": K * full.shape[1] / tc, "unit": "edges/s", "cores": threads,
                         "sample": f"all {full.shape[1]} C2 edges, K={K} d={d}: gcn_norm-weighted CSR built once, "
                                   f"torch.sparse.mm per layer + layer mean, median of 3"},
            "sample": f"random {frac:.0%} of the C2 edges ({ei.shape[1]} edges, all {graph.num_nodes} nodes), "
                      f"K={K} d={d} forward: index_select -> mul -> scatter_add_ with gcn_norm per layer "
                      f"(PyG 2.4.0 LGConv op sequence, torch {torch.__version__} CPU), median of {reps}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=["c2", "c5"], default="c2",
                    help="propagate workload: c2 = ML-25M-shaped K=3 d=64 (headline); c5 = 10M x 1M x 5e8, K=4 d=256")
    ap.add_argument("--layers", type=int, default=None, help="K (default 3 for c2, 4 for c5)")
    ap.add_argument("--dim", type=int, default=None, help="d (default 64 for c2, 256 for c5; train: 128)")
    ap.add_argument("--scale", type=float, default=1.0, help="graph scale vs ML-25M (1.0 = C2)")
    ap.add_argument("--chunk", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workload", choices=["propagate", "train"], default="propagate",
                    help="propagate: C2 headline (default); train: C3/C4 Cluster-GCN training steps")
    ap.add_argument("--parts", type=int, default=1024, help="train: Cluster-GCN parts")
    ap.add_argument("--parts-per-batch", type=int, default=32, help="train: parts per step")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) for runs; gloo to rehearse N ranks on one GPU")
    ap.add_argument("--torch-adam", action="store_true", help="train: torch Adam + clip_grad_norm_ (reference ops)")
    ap.add_argument("--no-graphs", action="store_true", help="train: run the fused step eagerly (no hipGraph replay)")
    ap.add_argument("--exchange", action="store_true",
                    help="train, N=1: run the row exchange anyway (measures its kernels; N>1 always uses it)")
    ap.add_argument("--dense-adam", action="store_true",
                    help="train: dense FusedAdam over all rows every step instead of the row-lazy exact Adam")
    ap.add_argument("--autograd", action="store_true",
                    help="train: reference-style step (compute_embeddings + bpr_loss + autograd) instead of "
                         "the fused no-autograd step")
    args = ap.parse_args()
    if args.workload == "train":
        return run_train(args)

    import numpy as np
    import torch
    import torch.distributed as dist

    import lgcn_amd
    from lgcn_amd import synth
    from lgcn_amd.plan import DEFAULT_CHUNK, PropagationPlan

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    dev = torch.device("cuda", local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    distributed = world > 1
    if distributed:
        init_dist(args.dist_backend, dev)

    c5 = args.config == "c5"
    K = args.layers if args.layers is not None else (4 if c5 else 3)
    d = args.dim if args.dim is not None else (256 if c5 else 64)
    d_full = d
    t0 = time.perf_counter()
    graph = None
    if c5:
        # C5: one synthetic 10M x 1M x 5e8-edge graph (same seed on every rank, generated on the GPU).
        # N > 1 ranks shard the embedding COLUMNS (feature-sharded propagation): every
        # rank runs the full plan on d/W columns, no collective; value = K*E / time (strong scaling).
        s = args.scale
        U, I = int(synth.C5_USERS * s), int(synth.C5_ITEMS * s)
        ei = synth.bipartite_device(U, I, int(synth.C5_PAIRS * s), seed=0, device=dev)
        if d % world or (d // world) % 4:
            raise SystemExit(f"c5 feature sharding needs d % (4*W) == 0 (d={d}, W={world})")
        d = d // world
        N, E = U + I, int(ei.shape[1])
        log(f"[rank {rank}] c5 graph U={U} I={I} E={E} on device, d={d_full} -> {d} columns per rank "
            f"({time.perf_counter() - t0:.1f} s)")
    else:
        graph = synth.ml25m_shaped(seed=rank, scale=args.scale)
        log(f"[rank {rank}] graph U={graph.num_users} I={graph.num_items} E={graph.num_edges} "
            f"{graph.degree_stats()} ({time.perf_counter() - t0:.1f} s)")
        U, I, N, E = graph.num_users, graph.num_items, graph.num_nodes, graph.num_edges
        ei = torch.from_numpy(graph.edge_index).to(dev)
    gen = torch.Generator(device=dev).manual_seed(rank)
    user_w = (torch.randn(U, d, device=dev, generator=gen) * 0.01).contiguous()
    item_w = (torch.randn(I, d, device=dev, generator=gen) * 0.01).contiguous()
    t0 = time.perf_counter()
    # side_split = U: rows gathering the item table run first, then rows gathering the user table
    plan = PropagationPlan(ei, N, args.chunk or DEFAULT_CHUNK, side_split=U)
    # the schedule the forward runs at this width: source-sliced (one lgcn_spmm_run launch per
    # slice per layer) when lgcn_amd.plan.slice_bytes_for enables it, else the plain item list
    from lgcn_amd.sliced import SlicedDirection

    sched = plan.schedule("fwd", d)
    n_slices = sum(1 for _, n in sched.launches if n) if isinstance(sched, SlicedDirection) else 1
    torch.cuda.synchronize()
    log(f"[rank {rank}] plan: {plan.fwd.n_items} items, {plan.fwd.n_splits} split rows, "
        f"{plan.fwd.n_partials} partials, {plan.nbytes() / 1e6:.0f} MB; "
        f"{n_slices} source slice(s) per layer, {sched.n_splits} chunked rows ({time.perf_counter() - t0:.2f} s)")

    def step():
        return lgcn_amd.propagate_forward(user_w, item_w, plan, K)

    with torch.no_grad():
        for _ in range(args.warmup):
            step()
        timer = LaunchTimer()
        lgcn_amd.set_launch_timer(timer)
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()
        timer.active = True
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        timer.active = False
        lgcn_amd.set_launch_timer(None)

    # the timer brackets each layer's item pass: n_slices launches (+ the short gaps between them)
    kernel_ms = timer.mean_ms() / n_slices
    edges_total = E
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        e = torch.tensor([E], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.SUM)
        edges_total = int(e.item())
        km = torch.tensor([kernel_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(km, op=dist.ReduceOp.MAX)
        kernel_ms = float(km.item())

    if c5:
        edges_total = E  # feature-sharded: the ranks together propagate one graph
    value = K * edges_total * args.steps / elapsed
    # algorithmic bytes of one layer, spread over the layer's n_slices launches
    bytes_per_layer = E * (4 * d + 8) + N * (4 * d + 8)
    bytes_per_launch = bytes_per_layer / n_slices
    achieved = bytes_per_launch / (kernel_ms * 1e-3) / 1e9
    if c5:
        workload = f"C5_synthetic_10Mx1M_5e8_K{K}_d{d_full}" + ("" if args.scale == 1.0 else f"_scale{args.scale}")
    else:
        workload = f"C2_ml25m_shaped_K{K}_d{d}" + ("" if args.scale == 1.0 else f"_scale{args.scale}")
    traffic = load_traffic(workload)
    result = {
        "metric": f"edges propagated/sec (K={K}, d={d_full})",
        "value": value,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if c5 else "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": ("synthetic (seeded 10M x 1M Zipf bipartite graph generated on device; random N(0,0.01) embeddings)"
                 if c5 else "synthetic (seeded ML-25M-shaped bipartite graph per rank; random N(0,0.01) embeddings)"),
        "config": {"workload": workload, "num_users": U, "num_items": I, "num_edges": E, "layers": K, "dim": d_full,
                   "chunk": plan.chunk, "graphs": 1 if c5 else world,
                   "parallelism": (f"feature-sharded over {world} GPU(s): {d} columns each, full plan per rank, "
                                   "no collective") if c5 else
                                  f"replicas: {world} independent graph instance(s), one per GPU, no collective"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": (f"k_spmm_vec<{kernel_lpr(d)},sliced> (lgcn_spmm_run, {n_slices} source-slice "
                                f"launches per layer)" if n_slices > 1 else
                                f"k_spmm_vec<{kernel_lpr(d)}> (lgcn_spmm_items)"),
                     "kernel_ms": kernel_ms, "bytes_per_launch": bytes_per_launch,
                     "launches_per_layer": n_slices},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not c5:
        result["cpu_baseline"] = cpu_baseline(graph, K, d)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


def run_train(args):
    """C3 (1 GPU) / C4 (N GPUs): Cluster-GCN training of LightGCN K=3, d=128 on the ML-25M-shaped
    graph: 90/5/5 directed split, train graph cut into --parts parts by the host LDG partitioner,
    --parts-per-batch parts per step (union of intra-part edges), BPR loss, backward through the
    HIP propagation, clip_grad_norm_(1), Adam(1e-3). N ranks = data parallel: disjoint batches per
    rank; with the default row-lazy Adam the ranks all_gather only their nonzero gradient rows
    (lgcn_amd.distributed.RowExchange); --dense-adam all_reduces both dense gradient tables.
    value = K * (batch edges summed over ranks) / wall time."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from data.dataset_handler import Data
    from lgcn_amd import cluster, synth
    from lgcn_amd import distributed as D
    from models.light_gcn import LightGCN
    from utils.train_test import bpr_loss, compute_embeddings

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if world > 1:
        init_dist(args.dist_backend, dev)
    K = args.layers if args.layers is not None else 3
    d = args.dim if args.dim is not None else 128
    t0 = time.perf_counter()
    g = synth.ml25m_shaped(seed=0, scale=args.scale)  # one graph, replicated tables (DP)
    U, I, N = g.num_users, g.num_items, g.num_nodes
    rng = np.random.default_rng(0)
    perm = rng.permutation(g.num_edges)
    n_tr = int(0.9 * g.num_edges)
    train_ei = np.ascontiguousarray(g.edge_index[:, np.sort(perm[:n_tr])])
    part = cluster.partition_nodes(train_ei, N, args.parts)
    f_intra = cluster.intra_fraction(train_ei, part)
    lists = cluster.intra_part_edges(train_ei, part, args.parts)
    order = np.random.default_rng(1).permutation(args.parts)
    q = args.parts_per_batch
    batches = []
    for b in range(0, args.parts, q):
        ei = np.concatenate([lists[p] for p in order[b:b + q]], axis=1)
        batches.append(Data(edge_index=torch.from_numpy(ei).to(dev), num_nodes=N))
    log(f"[rank {rank}] train graph E={n_tr} parts={args.parts} f_intra={f_intra:.4f} "
        f"batches={len(batches)} mean E_batch={np.mean([b.edge_index.shape[1] for b in batches]):.0f} "
        f"({time.perf_counter() - t0:.1f} s)")
    torch.manual_seed(0)
    model = LightGCN(U, I, num_layers=K, dim_h=d).to(dev)
    lazy = not (args.autograd or args.torch_adam or args.dense_adam)
    if args.torch_adam:
        opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    elif lazy:
        from lgcn_amd.optim import RowLazyAdam

        opt = RowLazyAdam(model.user_embedding.weight.data, model.item_embedding.weight.data, lr=1e-3,
                          max_grad_norm=1)
    else:
        from lgcn_amd.optim import FusedAdam

        opt = FusedAdam(model.parameters(), lr=1e-3, max_grad_norm=1, capturable=not args.autograd,
                        keep_clipped_grad=False)
    params = list(model.parameters())
    torch.manual_seed(1000 + rank)

    fused = None
    exchange = None
    if lazy and (world > 1 or args.exchange):
        # row-sparse DP gradient exchange: all_gather of each rank's nonzero gradient rows
        cap = D.exchange_capacity(batches, U)
        exchange = D.RowExchange(cap, N, d, dev, world)
        log(f"[rank {rank}] row exchange: {cap} slots per rank, {cap * (4 * d + 8) / 1e6:.1f} MB sent per step "
            f"(dense all_reduce: {N * d * 4 / 1e6:.1f} MB)")
    if not args.autograd:
        from lgcn_amd.train_step import FusedTrainStep

        fused = FusedTrainStep(model, opt, world=world, graphs=not args.no_graphs and not args.torch_adam,
                               lazy=lazy, exchange=exchange)

    def step(bidx):
        batch = batches[bidx]
        if fused is not None:
            fused.step(batch)
            return batch.edge_index.shape[1]
        opt.zero_grad()
        loss = bpr_loss(*compute_embeddings(model, batch, dev))
        loss.backward()
        D.allreduce_grads(params, world)
        if args.torch_adam:
            torch.nn.utils.clip_grad_norm_(params, max_norm=1)
        opt.step()
        return batch.edge_index.shape[1]

    share = D.rank_share(len(batches), world, rank, seed=0, epoch=0)
    for i in range(max(args.warmup, 2 * len(share))):  # warm-up builds every batch's plan
        step(share[i % len(share)])
        if fused is not None and (i + 1) % len(share) == 0:
            fused.sync()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    edges = 0
    for i in range(args.steps):
        edges += step(share[i % len(share)])
        # row-lazy Adam: parameters are made current once per epoch (as evaluation needs them),
        # inside the timed region
        if fused is not None and ((i + 1) % len(share) == 0 or i + 1 == args.steps):
            fused.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if fused is not None:
        fused.check_overflow()  # outside the timed region: one host read per batch state
    if world > 1:
        t = torch.tensor([elapsed, edges], dtype=torch.float64, device=dev)
        tt = t.clone()
        dist.all_reduce(t[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(tt[1:], op=dist.ReduceOp.SUM)
        elapsed, edges = float(t[0].item()), float(tt[1].item())
    result = {
        "metric": f"training edges propagated/sec (Cluster-GCN, K={K}, d={d})",
        "value": K * edges / elapsed, "unit": "edges/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (seeded ML-25M-shaped graph, 90/5/5 directed split)",
        "config": {"workload": f"C{3 if world == 1 else 4}_cluster_gcn_train", "parts": args.parts,
                   "optimizer": ("torch Adam + clip_grad_norm_" if args.torch_adam else
                                 "lgcn RowLazyAdam (exact row-lazy Adam + clip, flushed each epoch)" if lazy else
                                 "lgcn FusedAdam (clip fused)"),
                   "step": "autograd (reference ops)" if args.autograd else
                           ("fused sparse step" + ("" if (args.no_graphs or args.torch_adam) else ", hipGraph per batch")),
                   "parts_per_batch": q, "f_intra": f_intra, "layers": K, "dim": d, "num_users": U,
                   "num_items": I, "train_edges": n_tr,
                   "parallelism": (f"dp{world}: disjoint part batches per rank, " +
                                   ("row-sparse gradient exchange (all_gather of each rank's nonzero rows), "
                                    "row-lazy Adam on the union" if exchange is not None else
                                    "RCCL all_reduce of embedding grads" if world > 1 else "single GPU"))},
    }
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
