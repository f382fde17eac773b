"""Probe: where evaluate() (reference utils/train_test.py:136-212) spends its time at C3 scale.

python tools/eval_probe.py [--dim 128] [--layers 3]
Builds the ML-25M-shaped graph's 5 % validation edge set, then times evaluate()'s pieces on the
GPU: the forward over the val edges, the triplet gathers + bpr_loss, and compute_recall_at_k.
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "movie-recommender-system-with-gnns_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ties", default="index", help="lgcn_amd.tuning recall_ties: index | cpu")
    args = ap.parse_args()
    from lgcn_amd import synth, tuning

    tuning.set_tuning(recall_ties=args.ties)
    from models.light_gcn import LightGCN
    from utils import train_test as T

    g = synth.ml25m_shaped(seed=0)
    U, I = g.num_users, g.num_items
    E = g.num_edges
    perm = np.random.default_rng(0).permutation(E)
    val = np.sort(perm[int(0.9 * E):int(0.95 * E)])
    dev = torch.device("cuda")
    ei = torch.from_numpy(g.edge_index[:, val]).to(dev)

    class D:
        edge_index = ei

        def to(self, _):
            return self

    model = LightGCN(U, I, num_layers=args.layers, dim_h=args.dim).to(dev)

    def timed(fn):
        torch.cuda.synchronize()
        t = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        return out, (time.perf_counter() - t) * 1e3

    for _ in range(2):
        T.evaluate(model, D(), dev, top_k=100)
    for r in range(args.reps):
        with torch.no_grad():
            embs, t_emb = timed(lambda: T.compute_embeddings(model, D(), dev))
            _, t_loss = timed(lambda: T.bpr_loss(*embs).item())
            np.random.seed(r)
            rec, t_rec = timed(lambda: T.compute_recall_at_k((embs[1], embs[3], embs[5]), k=100))
        _, t_eval = timed(lambda: T.evaluate(model, D(), dev, top_k=100))
        print(f"ties={args.ties} E_val={ei.shape[1]} B={embs[0].shape[0]} d={args.dim}: embeddings {t_emb:.2f} ms, "
              f"loss {t_loss:.2f} ms, recall@100 {t_rec:.2f} ms (={rec:.3e}), evaluate {t_eval:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
