"""Projection of C4 (Cluster-GCN training, K=3, d=128, 1024 parts, 32 parts per batch) to W ranks
of one node, per --dp-mode, from one GPU (the C2 counterpart is
tools/project_scale.py). Every piece of a rank's step is timed on this GPU; the collectives are
priced from a bus bandwidth and a latency per collective, which a one-GPU box cannot measure.

  columns     every rank steps the one-GPU schedule (the same batches, negatives, Adam steps) on
              d/W columns: the one-GPU step at width d/W, plus one all_reduce of the triplets'
              [B, 6] dots / norms and one all_gather of the clip norm's partials per step. Strong
              scaling: speed-up = T_1(d) / step_W.
  replicated  data parallel over disjoint parts: each rank's own gradient step (T_1 with the
              exchange's pack kernels) + one all_gather of every rank's record block + the row
              Adam on the UNION of the W batches' rows (timed by emulation: the W ranks' blocks
              computed one after another on this GPU, then the union update timed alone) + the
              per-epoch flush (32 / W steps per epoch). Weak: speed-up = W T_1(d) / step_W.
  hybrid      the replicated step with the item gradient table all_reduced densely (ring) and only
              the users' rows all-gathered; every item row stepped each step (update timed by
              emulation with W ranks' user blocks). Weak.
  owner       the replicated step with the union update shared by the W owners (each owner
              updates 1/W of the union: the replicated union update / W, a lower bound) and two
              all_to_alls of (W-1)/W of its blocks instead of the all_gather, plus the per-epoch
              all_gather of the owned rows.

python tools/project_c4.py [--graph ml25m|planted] [--worlds 2,4,8] [--busbw 50,100,200] [--lat-us 20]"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "movie-recommender-system-with-gnns_amd"))
sys.path.insert(0, ROOT)


class _B:
    def __init__(self, ei):
        self.edge_index = ei


def _ev():
    return torch.cuda.Event(enable_timing=True)


def one_gpu_step_ms(U, I, d, batches, exchange=False, epochs=3):
    """ms per step of the fused lazy step over whole epochs of the batches (graphs, flush once per
    epoch inside the timed region) at width d, the bench's C3 loop; with exchange=True the W = 1
    row exchange runs too (its pack / mark / accumulate kernels); exchange="hybrid": the W = 1
    HybridExchange (the item gradient table zeroed each step, the users packed, every item row
    stepped)."""
    from lgcn_amd import distributed as D
    from lgcn_amd.optim import RowLazyAdam
    from lgcn_amd.train_step import FusedTrainStep
    from models.light_gcn import LightGCN

    torch.manual_seed(0)
    dev = batches[0].edge_index.device
    m = LightGCN(U, I, num_layers=3, dim_h=d).to(dev)
    opt = RowLazyAdam(m.user_embedding.weight.data, m.item_embedding.weight.data, lr=1e-3, max_grad_norm=1,
                      max_steps=4096)
    if exchange == "hybrid":
        ex = D.HybridExchange(D.user_exchange_capacity(batches, U), U, opt.gi, dev, 1)
    else:
        ex = D.RowExchange(D.exchange_capacity(batches, U), U + I, d, dev, 1) if exchange else None
    step = FusedTrainStep(m, opt, graphs=True, lazy=True, exchange=ex)
    for _ in range(2):  # warm-up epochs: plans built, graphs captured
        for b in batches:
            step.step(b)
        step.sync()
    torch.cuda.synchronize()
    a, z = _ev(), _ev()
    a.record()
    for _ in range(epochs):
        for b in batches:
            step.step(b)
        step.sync()
    z.record()
    torch.cuda.synchronize()
    return a.elapsed_time(z) / (epochs * len(batches))


def union_update_ms(U, I, d, batches, W, reps=6):
    """The replicated exchange's update on the union of W ranks' rows (mark first + rank-order sum
    + clip norm + row Adam), timed alone: the W blocks are computed one after another on this GPU
    (each rank's _lazy_grads for its own batch), copied into the all-gathered buffer, then
    _lazy_update runs once — what every rank runs after the all_gather. Also returns the own-rows
    update (W = 1) for the same step structure."""
    from lgcn_amd import distributed as D
    from lgcn_amd.optim import RowLazyAdam
    from lgcn_amd.train_step import FusedTrainStep
    from models.light_gcn import LightGCN

    torch.manual_seed(0)
    dev = batches[0].edge_index.device
    m = LightGCN(U, I, num_layers=3, dim_h=d).to(dev)
    opt = RowLazyAdam(m.user_embedding.weight.data, m.item_embedding.weight.data, lr=1e-3, max_grad_norm=1,
                      max_steps=4096)
    cap = D.exchange_capacity(batches, U)
    ex = D.RowExchange(cap, U + I, d, dev, W)
    step = FusedTrainStep(m, opt, world=W, graphs=False, lazy=True, exchange=ex)
    order = np.random.default_rng(0).permutation(len(batches))
    ts = []
    k = 0
    for rep in range(reps + 2):
        group = [batches[order[(k + r) % len(batches)]] for r in range(W)]
        k += W
        with torch.no_grad():
            for r, b in enumerate(group):
                st = step.state(b.edge_index)
                step._lazy_grads(st)
                ex.pack_all.view(W, ex.blk)[r].copy_(ex.pack)
        torch.cuda.synchronize()
        a, z = _ev(), _ev()
        a.record()
        step._lazy_update(st)
        z.record()
        torch.cuda.synchronize()
        if rep >= 2:
            ts.append(a.elapsed_time(z))
    a, z = _ev(), _ev()
    a.record()
    step.sync()  # the per-epoch flush: every deferred row replayed up to date
    z.record()
    torch.cuda.synchronize()
    return float(np.median(ts)), ex.blk * 4, a.elapsed_time(z)


def hybrid_update_ms(U, I, d, batches, W, reps=6):
    """HybridExchange's update on W ranks' user records (emulated as union_update_ms does) plus
    every item row: mark first + the users' rank-order sums + the item table / W + clip norm + row
    Adam on all items and the union of the users."""
    from lgcn_amd import distributed as D
    from lgcn_amd.optim import RowLazyAdam
    from lgcn_amd.train_step import FusedTrainStep
    from models.light_gcn import LightGCN

    torch.manual_seed(0)
    dev = batches[0].edge_index.device
    m = LightGCN(U, I, num_layers=3, dim_h=d).to(dev)
    opt = RowLazyAdam(m.user_embedding.weight.data, m.item_embedding.weight.data, lr=1e-3, max_grad_norm=1,
                      max_steps=4096)
    ex = D.HybridExchange(D.user_exchange_capacity(batches, U), U, opt.gi, dev, W)
    step = FusedTrainStep(m, opt, world=W, graphs=False, lazy=True, exchange=ex)
    order = np.random.default_rng(0).permutation(len(batches))
    ts = []
    k = 0
    for rep in range(reps + 2):
        group = [batches[order[(k + r) % len(batches)]] for r in range(W)]
        k += W
        with torch.no_grad():
            for r, b in enumerate(group):
                st = step.state(b.edge_index)
                step._lazy_grads(st)
                ex.pack_all.view(W, ex.blk)[r].copy_(ex.pack)
        torch.cuda.synchronize()
        a, z = _ev(), _ev()
        a.record()
        step._lazy_update(st)
        z.record()
        torch.cuda.synchronize()
        if rep >= 2:
            ts.append(a.elapsed_time(z))
    return float(np.median(ts)), ex.blk * 4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", choices=["ml25m", "planted"], default="ml25m")
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--busbw", default="50,100,200")
    ap.add_argument("--lat-us", type=float, default=20.0)
    ap.add_argument("--dim", type=int, default=128)
    args = ap.parse_args()
    from lgcn_amd import cluster, synth
    from lgcn_amd.owner import owner_capacity

    dev = torch.device("cuda")
    g = synth.planted_ml25m(1024)[0] if args.graph == "planted" else synth.ml25m_shaped(seed=0)
    U, I, N = g.num_users, g.num_items, g.num_nodes
    train = synth.train_split(g.edge_index, 0.9, seed=0)
    _, f_intra, lists = cluster.cluster_batches(train, N, 1024, 32)
    batches = [_B(torch.from_numpy(x).to(dev)) for x in lists]
    d = args.dim
    B_mean = float(np.mean([int((x[0] < U).sum()) for x in lists]))
    E_mean = float(np.mean([x.shape[1] for x in lists]))
    worlds = [int(w) for w in args.worlds.split(",")]
    lat = args.lat_us / 1e3
    t1 = one_gpu_step_ms(U, I, d, batches)
    t1x = one_gpu_step_ms(U, I, d, batches, exchange=True)
    upd1, _, flush = union_update_ms(U, I, d, batches, 1)
    t1h = one_gpu_step_ms(U, I, d, batches, exchange="hybrid")
    upd1h, _ = hybrid_update_ms(U, I, d, batches, 1)
    print(f"C4 projection, {args.graph} graph: {len(batches)} batches of {E_mean:.0f} edges (B {B_mean:.0f} "
          f"triplets), f_intra {f_intra:.4f}, K=3 d={d}. One GPU: {t1:.4f} ms per step ({3 * E_mean / t1 / 1e6:.3g}e9 "
          f"edges/s); with the W=1 row exchange {t1x:.4f} ms, with the W=1 hybrid exchange {t1h:.4f} ms; own-rows "
          f"update {upd1 * 1e3:.1f} us (hybrid {upd1h * 1e3:.1f}); per-epoch flush {flush * 1e3:.1f} us", flush=True)
    for W in worlds:
        if d % W or (d // W) % 4:
            continue
        tc = one_gpu_step_ms(U, I, d // W, batches)
        updW, blk_bytes, _ = union_update_ms(U, I, d, batches, W)
        updWh, hblk_bytes = hybrid_update_ms(U, I, d, batches, W)
        # T_1 carries one flush per 32 steps; a W-rank epoch is 32 / W steps
        extra_flush = flush * (1.0 / (len(batches) // W) - 1.0 / len(batches))
        spe = len(batches) // W  # steps per epoch (each step takes W batches)
        ocap = owner_capacity(batches, U, W, num_items=I)
        oblk = ocap * (d + 2) + 2 * ocap
        oblk += (-oblk) % 4
        owned_rows = -(-N // W)
        print(f" W={W}: columns rank step (d={d // W}) {tc:.4f} ms; union update {updW * 1e3:.1f} us "
              f"(own rows {upd1 * 1e3:.1f}); hybrid update {updWh * 1e3:.1f} us (own {upd1h * 1e3:.1f}); record "
              f"block {blk_bytes / 1e6:.2f} MB, owner block {oblk * 4 / 1e6:.2f} MB, hybrid user block "
              f"{hblk_bytes / 1e6:.2f} MB + items {I * d * 4 / 1e6:.1f} MB all_reduced", flush=True)
        for bw in (float(v) for v in args.busbw.split(",")):
            # columns: all_reduce of [B, 6] floats + all_gather of W x 2048 norm partials
            cols = tc + 2 * lat + (2 * (W - 1) / W * B_mean * 24 + (W - 1) * 2048 * 4) / 1e6 / bw
            # replicated: own step (with pack) + all_gather of (W-1) blocks + the union update's extra
            rep = t1x + lat + (W - 1) * blk_bytes / 1e6 / bw + (updW - upd1) + extra_flush
            # owner: two all_to_alls of (W-1)/W blocks + norm partials; union update shared by W owners;
            # the per-epoch all_gather of the owned rows spread over the epoch's steps
            own = (t1x + 3 * lat + (2 * (W - 1) * oblk * 4 + (W - 1) * 2048 * 4) / 1e6 / bw + (updW / W - upd1 / W)
                   + (lat + (W - 1) * owned_rows * d * 4 / 1e6 / bw) / spe)
            # hybrid: own step (zeroed item table, users packed, all items stepped) + the users' all_gather
            # + a ring all_reduce of the item gradient table + the union update's extra over the own one
            hyb = (t1h + 2 * lat + ((W - 1) * hblk_bytes + 2 * (W - 1) / W * I * d * 4) / 1e6 / bw
                   + (updWh - upd1h) + extra_flush)
            print(f"   busbw {bw:.0f} GB/s (+{args.lat_us:.0f} us each): columns {cols:.4f} ms ({t1 / cols:.2f}x) | "
                  f"replicated {rep:.4f} ms ({W * t1 / rep:.2f}x) | owner {own:.4f} ms ({W * t1 / own:.2f}x) | "
                  f"hybrid {hyb:.4f} ms ({W * t1 / hyb:.2f}x)", flush=True)


if __name__ == "__main__":
    main()
