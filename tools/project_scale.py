"""Projection of the reduce-mode C2 grid (lgcn_amd.sharded, users sharded, item partials all-reduced
per layer) to a node of R x F GPUs, from one GPU: each piece of a rank's K=3 step is timed alone
(HIP events, the rank's own plans, the heavier of row groups 0 and R-1), then the step is replayed
as an event schedule with the per-layer all_reduce / last-layer reduce_scatter priced from a bus
bandwidth and a latency that this box cannot measure (one GPU per box). Two orders:

  overlapped: P_k (+ its combine) -> all_reduce_k starts; U_k (+ combine) waits for all_reduce_{k-1}
              (P_k needs U_{k-1}); all_reduce_k overlaps U_k and P_{k+1}.
  fused:      pair_k = P_k and U_k in one launch (+ one combine launch), then all_reduce_k; pair_{k+1}
              waits for it.

  chunked:    the overlapped order with P_k issued as B item-row blocks, block b's all_reduce (or,
              at k = K, its reduce_scatter) started on the side stream as soon as the block is summed
              (VERDICT r4 item 1), each collective paying the latency term: AR_k overlaps P_k's own
              tail as well as U_k + P_{k+1}, and the last layer's reduce_scatter no longer waits for
              the whole P_K.

Every order also obeys a closed-form floor: the collectives of one step run one after another on
their stream and the first cannot start before some of P_1 is summed, so
    step >= t_P / B + (K-1) (B lat + AR bytes / busbw) + (B lat + RS bytes / busbw)
whatever the overlap; `--pieces-us` prices from recorded pieces (no GPU needed).

python tools/project_scale.py [--grids 8x1,4x2] [--busbw 100,150,200,300] [--lat-us 15] [--blocks 1,2,4]
python tools/project_scale.py --pieces-us 4x2:32.3,33.4,60.2 --one-gpu-ms 1.2154   (CPU: price only)"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "movie-recommender-system-with-gnns_amd"))

from lgcn_amd import _ffi, synth  # noqa: E402
from lgcn_amd.sharded import ReducePlan, ShardGrid, UserShards  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from scale_model import simulate  # noqa: E402,F401  (the shared event model)


def timed(fn, reps=30):
    """mean ms of fn() over reps (events on the current stream, after 3 warm-ups)."""
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def pieces(rplan, x0u, x0i, d):
    """ms of: the partial pass, the user pass, their pair launch (items + combines) — each a
    middle-layer (ADD) launch set on layer-0-shaped tables."""
    U, dev = x0u.shape[0], x0u.device
    I_pad = rplan.I_pad
    part = torch.zeros((I_pad, d), device=dev)
    acc_u = torch.zeros((U, d), device=dev)
    y = torch.empty((U, d), device=dev)
    acc = (acc_u, torch.zeros((x0i.shape[0], d), device=dev), U)
    t_p = timed(lambda: rplan.run_partial(x0u, part))
    t_u = timed(lambda: rplan.run_users(x0i, None, acc, y, _ffi.EPI_ADD, 1.0, 1.0))
    t_pair = timed(lambda: rplan.run_pair(x0u, part, x0i, None, acc, y, _ffi.EPI_ADD, 1.0, 1.0))
    return t_p, t_u, t_pair


def simulate_chunked(K, t_p, t_u, t_ar, t_rs, blocks, lat, t_block=0.0):
    """The overlapped order with P_k cut into `blocks` item-row blocks (each t_p / blocks + t_block
    of compute, t_block = the extra launch and tail per block) and one collective per block as soon
    as it is summed; t_ar / t_rs are the bandwidth terms of a whole table's all_reduce /
    reduce_scatter, lat the latency of each collective. blocks = 1 is `simulate(..., fused=False)`."""
    t, comm, ar_done = 0.0, 0.0, {0: 0.0}
    for k in range(1, K + 1):
        for _ in range(blocks):
            t += t_p / blocks + (t_block if blocks > 1 else 0.0)
            comm = max(comm, t) + lat + (t_ar if k < K else t_rs) / blocks
        ar_done[k] = comm
        t = max(t, ar_done[k - 1]) + t_u  # U_k reads every item row reduced one layer earlier
    return max(t, ar_done[K])


def comm_floor(K, t_p, t_ar, t_rs, blocks, lat):
    """The step can end no earlier than its serial collectives, which start after P_1's first block."""
    return t_p / blocks + (K - 1) * (blocks * lat + t_ar) + blocks * lat + t_rs


def price(name, R, K, t_p, t_u, t_pair, mb, args, stack_ms=0.005):
    """Print the projection table of one grid from its pieces (ms) and its item table (MB)."""
    print(f"grid {name} (R={R}): partial pass {t_p * 1e3:.1f} us, user pass {t_u * 1e3:.1f} us, "
          f"pair {t_pair * 1e3:.1f} us (vs {1e3 * (t_p + t_u):.1f} us apart); item table {mb:.1f} MB", flush=True)
    lat = args.lat_us / 1e3
    for bw in (float(v) for v in args.busbw.split(",")):
        # ring all_reduce: 2 (R-1)/R of the table over the bus bandwidth; reduce_scatter half of it
        a, r = 2 * (R - 1) / R * mb / bw, (R - 1) / R * mb / bw  # MB / (GB/s) = ms
        o = simulate(K, t_p, t_u, t_pair, lat + a, lat + r, False) + stack_ms
        f = simulate(K, t_p, t_u, t_pair, lat + a, lat + r, True) + stack_ms
        c = K * (t_p + t_u) + stack_ms
        line = (f"  busbw {bw:.0f} GB/s (+{args.lat_us:.0f} us): all_reduce {(lat + a) * 1e3:.0f} us; overlapped "
                f"{o:.3f} ms ({args.one_gpu_ms / o:.2f}x), fused {f:.3f} ms ({args.one_gpu_ms / f:.2f}x)")
        for B in (int(v) for v in args.blocks.split(",")):
            if B > 1:
                ch = simulate_chunked(K, t_p, t_u, a, r, B, lat, args.block_us / 1e3) + stack_ms
                line += f", chunked B={B} {ch:.3f} ms ({args.one_gpu_ms / ch:.2f}x)"
        fl = comm_floor(K, t_p, a, r, 1, lat) + stack_ms
        line += (f"; compute alone {c:.3f} ms ({args.one_gpu_ms / c:.2f}x); exchange floor {fl:.3f} ms "
                 f"(<= {args.one_gpu_ms / fl:.2f}x)")
        print(line, flush=True)
    # the bus bandwidth below which no order reaches `target`x: the floor at B = 1 (chunking only
    # adds latency terms to it) must fit the target step
    target = args.one_gpu_ms / args.target
    room = target - stack_ms - t_p - K * lat
    need = (2 * (K - 1) + 1) * (R - 1) / R * mb / room if room > 0 else float("inf")
    print(f"  {args.target:.0f}x needs a step <= {target * 1e3:.0f} us: exchange floor -> busbw >= {need:.0f} GB/s "
          f"(any order, any B); compute alone {K * (t_p + t_u) + stack_ms:.3f} ms", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grids", default="8x1,4x2")
    ap.add_argument("--busbw", default="100,150,200,300")
    ap.add_argument("--lat-us", type=float, default=15.0)
    ap.add_argument("--one-gpu-ms", type=float, default=1.2154,
                    help="the one-GPU K=3 step (round 5, the driver's command with the settled warm-up, profiles/r05b_settle)")
    ap.add_argument("--blocks", default="1,2,4", help="item-row blocks of the chunked order")
    ap.add_argument("--block-us", type=float, default=3.0, help="extra launch + tail per block (chunked order)")
    ap.add_argument("--target", type=float, default=6.0)
    ap.add_argument("--pieces-us", default=None,
                    help="RxF:P,U,PAIR[;RxF:...]: price recorded pieces (us) instead of timing them (no GPU)")
    args = ap.parse_args()
    K, d_full, I = 3, 64, 59047
    if args.pieces_us:
        for spec in args.pieces_us.split(";"):
            name, vals = spec.split(":")
            R, F = (int(v) for v in name.split("x"))
            t_p, t_u, t_pair = (float(v) / 1e3 for v in vals.split(","))
            price(name, R, K, t_p, t_u, t_pair, (-(-I // R) * R) * (d_full // F) * 4 / 1e6, args)
        return
    dev = torch.device("cuda")
    g = synth.ml25m_shaped(seed=0)
    U, I, N = g.num_users, g.num_items, g.num_nodes
    ei = torch.from_numpy(g.edge_index).to(dev)
    deg = np.bincount(g.edge_index[1], minlength=N)
    gen = torch.Generator(device=dev).manual_seed(0)
    uw = torch.randn(U, d_full, device=dev, generator=gen) * 0.01
    iw = torch.randn(I, d_full, device=dev, generator=gen) * 0.01
    for spec in args.grids.split(","):
        R, F = (int(v) for v in spec.split("x"))
        grid = ShardGrid.build(R * F, 0, d_full, R, F)
        c0, c1 = grid.cols
        d = c1 - c0
        shards = UserShards.build(deg, U, R)
        worst = None
        for gr in sorted({0, R - 1}):
            rplan = ReducePlan(ei, shards, gr, d)
            x0u, x0i = uw[:, c0:c1].contiguous(), iw[:, c0:c1].contiguous()
            p = pieces(rplan, x0u, x0i, d)
            worst = p if worst is None or sum(p) > sum(worst) else worst
            del rplan
        t_p, t_u, t_pair = worst
        price(f"{R}x{F}", R, K, t_p, t_u, t_pair, (-(-I // R) * R) * d * 4 / 1e6, args)


if __name__ == "__main__":
    main()
