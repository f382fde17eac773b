"""Diagnostic: dense FusedTrainStep+FusedAdam vs lazy FusedTrainStep+RowLazyAdam, step by step."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "movie-recommender-system-with-gnns_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import graphs  # noqa: E402
from lgcn_amd import cluster as C  # noqa: E402
from lgcn_amd.optim import FusedAdam, RowLazyAdam  # noqa: E402
from lgcn_amd.train_step import FusedTrainStep  # noqa: E402
from models.light_gcn import LightGCN  # noqa: E402


class B:
    def __init__(self, e):
        self.edge_index = e


gpu = torch.device("cuda")
U, I, ei = graphs.subsampled(U=2000, I=1000, pairs=8000, seed=4)
part = C.partition_nodes(ei, U + I, 8)
batches = [B(torch.from_numpy(x).to(gpu)) for x in C.intra_part_edges(ei, part, 8)]
models, steps, opts = [], [], []
for lazy in (False, True):
    torch.manual_seed(0)
    m = LightGCN(U, I, num_layers=3, dim_h=64).to(gpu)
    opt = (RowLazyAdam(m.user_embedding.weight.data, m.item_embedding.weight.data, lr=1e-2, max_grad_norm=None) if lazy
           else FusedAdam(m.parameters(), lr=1e-2, max_grad_norm=None, capturable=True))
    models.append(m)
    opts.append(opt)
    steps.append(FusedTrainStep(m, opt, lazy=lazy))
for i in range(6):
    b = batches[i % 8]
    torch.cuda.manual_seed(100 + i)
    la = steps[0].step(b).item()
    ga = torch.cat([models[0].user_embedding.weight.grad, models[0].item_embedding.weight.grad])
    torch.cuda.manual_seed(100 + i)
    lb = steps[1].step(b).item()
    gb = torch.cat([opts[1].gu, opts[1].gi])
    st = steps[1].state(b.edge_index)
    R = torch.zeros(U + I, dtype=torch.bool, device=gpu)
    R[st.touched_rows.long()] = True
    R[st.neg + U] = True
    gdiff = (ga[R] - gb[R]).abs().max().item()
    if i == 2:
        T = torch.zeros(U + I, dtype=torch.bool, device=gpu)
        T[st.touched_rows.long()] = True
        NG = torch.zeros(U + I, dtype=torch.bool, device=gpu)
        NG[st.neg + U] = True
        bad = (ga - gb).abs().max(1).values > 1e-7
        for nm, msk in (("touched&!neg", T & ~NG), ("touched&neg", T & NG), ("untouched neg", ~T & NG)):
            print(f"   {nm}: rows {int(msk.sum())}, bad {int((bad & msk).sum())}", flush=True)
        rb = torch.nonzero(bad & R).squeeze(1)[:5].tolist()
        for r in rb:
            print(f"   row {r}: dense {ga[r, :3].tolist()} lazy {gb[r, :3].tolist()} touched {bool(T[r])} neg {bool(NG[r])}",
                  flush=True)
    outside = ga[~R].abs().max().item()
    print(f"step {i}: loss {la:.6f} {lb:.6f}  grad diff on R {gdiff:.3e} (max {ga[R].abs().max().item():.3e}) "
          f"dense grad outside R {outside:.3e}  ",
          flush=True)
    # rows read by this step (touched + negatives) are current in the lazy model: compare them
    ua = torch.cat([models[0].user_embedding.weight, models[0].item_embedding.weight]).detach()
    ub = torch.cat([models[1].user_embedding.weight, models[1].item_embedding.weight]).detach()
    lastv = opts[1].last
    cur = lastv == opts[1].steps
    print(f"   rows current in lazy: {int(cur.sum())}, param diff on them {(ua[cur] - ub[cur]).abs().max().item():.3e}",
          flush=True)
    if False:
      for name, x, y in (("user", models[0].user_embedding.weight, models[1].user_embedding.weight),
                       ("item", models[0].item_embedding.weight, models[1].item_embedding.weight)):
        dd = (x.detach() - y.detach()).abs()
        print(f"   {name}: param diff max {dd.max().item():.3e} at row {int(dd.max(1).values.argmax())}", flush=True)
