"""Probe: source-sliced, XCD-queued schedule for the C2 item pass (prototype, built with torch ops).

Every row's edge list (sorted by source id) is cut at source-slice boundaries; slice s of a side
goes to XCD queue s % 8, so an XCD's L2 only ever holds its slices of the gathered table. Rows
with more than one (slice, chunk) item sum partials in the combine pass.
python tools/slice_probe.py [--slices-items 8] [--slices-users 16]
"""
import argparse
import copy
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "movie-recommender-system-with-gnns_amd"))

import lgcn_amd  # noqa: E402
from lgcn_amd import synth  # noqa: E402
from lgcn_amd.plan import CsrDirection, PropagationPlan  # noqa: E402


def sliced_direction(f: CsrDirection, N: int, U: int, S_user: int, S_item: int, chunk: int, gpb: int,
                     nxcd: int = 8) -> CsrDirection:
    dev = f.rowptr.device
    rowptr, col = f.rowptr, f.col.long()
    E = col.numel()
    I = N - U
    deg = rowptr[1:] - rowptr[:-1]
    row = torch.repeat_interleave(torch.arange(N, device=dev), deg)
    is_item = col >= U
    s = torch.where(is_item, S_user + ((col - U) * S_item) // I, (col * S_user) // U)  # global slice id
    # phase: item-source slices first (rows gathering the smaller item table), then user-source
    phase_key = torch.where(s >= S_user, s - S_user, S_item + s)
    start = torch.ones(E, dtype=torch.bool, device=dev)
    start[1:] = (row[1:] != row[:-1]) | (s[1:] != s[:-1])
    seg_id = torch.cumsum(start.long(), 0) - 1
    seg_beg = torch.nonzero(start).squeeze(1)
    nseg = seg_beg.numel()
    seg_len = torch.diff(torch.cat([seg_beg, torch.tensor([E], device=dev)]))
    seg_row = row[seg_beg]
    seg_s = s[seg_beg]
    seg_phase = phase_key[seg_beg]
    # chunks
    nch = (seg_len + chunk - 1) // chunk
    it_seg = torch.repeat_interleave(torch.arange(nseg, device=dev), nch)
    first = torch.cumsum(nch, 0) - nch
    it_c = torch.arange(it_seg.numel(), device=dev) - first[it_seg]
    it_beg = seg_beg[it_seg] + it_c * chunk
    it_len = torch.minimum(seg_len[it_seg] - it_c * chunk, torch.tensor(chunk, device=dev))
    it_row = seg_row[it_seg]
    it_q = seg_s[it_seg] % nxcd
    it_phase = seg_phase[it_seg]
    # empty rows: one len-0 item each (their epilogue still runs)
    empty = torch.nonzero(deg == 0).squeeze(1)
    it_beg = torch.cat([it_beg, torch.zeros_like(empty)])
    it_len = torch.cat([it_len, torch.zeros_like(empty)])
    it_row = torch.cat([it_row, empty])
    it_q = torch.cat([it_q, torch.zeros_like(empty)])
    it_phase = torch.cat([it_phase, torch.full_like(empty, 10 ** 6)])
    n = it_row.numel()
    # per-row item counts -> partial slots for rows with >= 2 items, in (slice, chunk) order
    cnt = torch.bincount(it_row, minlength=N)
    multi = cnt >= 2
    # order items by row then global position (already row-major, slices ascending, chunks ascending)
    order_row = torch.argsort(it_row * (E + 1) + it_beg, stable=True)
    pcnt = torch.where(multi, cnt, torch.zeros_like(cnt))
    pbeg = torch.cumsum(pcnt, 0) - pcnt
    n_partials = int(pcnt.sum())
    rank = torch.empty(n, dtype=torch.long, device=dev)
    rr = it_row[order_row]
    firsts = torch.cumsum(cnt, 0) - cnt
    rank[order_row] = torch.arange(n, device=dev) - firsts[rr]
    dst = torch.where(multi[it_row], -(pbeg[it_row] + rank) - 1, it_row)
    split_rows = torch.nonzero(multi).squeeze(1)
    splits = torch.stack([split_rows, pbeg[split_rows], pcnt[split_rows], torch.zeros_like(split_rows)], 1).int()
    # queues: within a queue, phase then longest first
    key = (it_q * 10 ** 7 + it_phase) * (chunk + 1) + (chunk - it_len)
    o = torch.argsort(key, stable=True)
    it_beg, it_len, dst, it_q = it_beg[o], it_len[o], dst[o], it_q[o]
    qlen = torch.bincount(it_q, minlength=nxcd)
    blocks_per_q = (qlen + gpb - 1) // gpb
    nb = int(blocks_per_q.max())
    total = nb * nxcd * gpb
    dummy = n_partials  # extra slot for padding items
    out_beg = torch.zeros(total, dtype=torch.long, device=dev)
    out_len = torch.zeros(total, dtype=torch.long, device=dev)
    out_dst = torch.full((total,), -(dummy + 1), dtype=torch.long, device=dev)
    qstart = torch.cumsum(qlen, 0) - qlen
    pos_in_q = torch.arange(n, device=dev) - qstart[it_q]
    blk = pos_in_q // gpb
    slot = (blk * nxcd + it_q) * gpb + pos_in_q % gpb
    out_beg[slot] = it_beg
    out_len[slot] = it_len
    out_dst[slot] = dst
    items = torch.empty((total, 2), dtype=torch.int64, device=dev)
    items[:, 0] = out_beg
    items[:, 1] = (out_len & 0xFFFFFFFF) | (out_dst << 32)
    return CsrDirection(f.rowptr, f.col, f.eid, f.val, items, splits.contiguous(), total, split_rows.numel(),
                        n_partials + 1, chunk), dict(items=n, blocks=nb * nxcd, pad=total - n, partials=n_partials,
                                                      splits=split_rows.numel(), qlen=qlen.tolist())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slices-items", type=int, default=8)
    ap.add_argument("--slices-users", type=int, default=16)
    ap.add_argument("--chunk", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda")
    g = synth.ml25m_shaped(seed=0)
    U, I, N = g.num_users, g.num_items, g.num_nodes
    ei = torch.from_numpy(g.edge_index).to(dev)
    K, d = 3, 64
    gen = torch.Generator(device=dev).manual_seed(0)
    uw = torch.randn(U, d, device=dev, generator=gen) * 0.01
    iw = torch.randn(I, d, device=dev, generator=gen) * 0.01
    plan = PropagationPlan(ei, N, 256, side_split=U)
    t0 = time.perf_counter()
    sl, info = sliced_direction(plan.fwd, N, U, args.slices_users, args.slices_items, args.chunk, 256 // (d // 4))
    torch.cuda.synchronize()
    print(f"sliced schedule built in {time.perf_counter() - t0:.2f} s: {info}", flush=True)
    plan2 = copy.copy(plan)
    plan2.fwd = sl

    def timeit(p, label):
        with torch.no_grad():
            for _ in range(3):
                out = lgcn_amd.propagate_forward(uw, iw, p, K)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(args.steps):
                out = lgcn_amd.propagate_forward(uw, iw, p, K)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t) / args.steps * 1e3
        print(f"{label:10s} {ms:.3f} ms/step  {K * g.num_edges / ms / 1e6:.2f} e9 edges/s", flush=True)
        return out

    for _ in range(2):
        a = timeit(plan, "default")
        b = timeit(plan2, "sliced")
    rel = ((a - b).abs().max(dim=1).values / a.abs().max(dim=1).values.clamp_min(1e-30)).max().item()
    print(f"max row-relative diff sliced vs default: {rel:.3e}", flush=True)


if __name__ == "__main__":
    main()
