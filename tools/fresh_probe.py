"""Where the harness's extra time per step goes when the loader collates new DEVICE tensors every
epoch (bench.py harness.fused_fresh_device_tensors vs fused): C3 batches, utils.train_test.train()
over one epoch (the second of two), four loaders:
  same     the same Data objects every epoch
  clone    a clone is made per batch (the loader's own cost) but the same object is yielded
  fresh    the clone is yielded (content keys by the device digest, prefetched one batch ahead)
  fresh-np the clone is yielded with the lookahead prefetch disabled (digest collected on demand)
python tools/fresh_probe.py"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "movie-recommender-system-with-gnns_amd"), ROOT]


def main():
    from data.dataset_handler import Data
    from lgcn_amd import _cache, cluster, harness, synth
    from models.light_gcn import LightGCN
    from utils import train_test as TT

    dev = torch.device("cuda")
    g = synth.ml25m_shaped(seed=0)
    train = synth.train_split(g.edge_index, 0.9, seed=0)
    _, _, lists = cluster.cluster_batches(train, g.num_nodes, 1024, 32)
    src = [torch.from_numpy(x).to(dev) for x in lists]
    same = [Data(edge_index=e, num_nodes=g.num_nodes) for e in src]

    class Loader:
        def __init__(self, kind):
            self.kind = kind

        def __len__(self):
            return len(src)

        def __iter__(self):
            for i, e in enumerate(src):
                if self.kind == "same":
                    yield same[i]
                elif self.kind == "clone":
                    e.clone()
                    yield same[i]
                else:
                    yield Data(edge_index=e.clone(), num_nodes=g.num_nodes)

    orig = _cache.prefetch
    for kind in ("same", "clone", "fresh", "fresh-np", "same"):
        _cache.prefetch = (lambda t: None) if kind == "fresh-np" else orig
        torch.manual_seed(0)
        m = LightGCN(g.num_users, g.num_items, num_layers=3, dim_h=128).to(dev)
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        loader = Loader("fresh" if kind.startswith("fresh") else kind)
        for e in range(3):
            torch.cuda.synchronize()
            t = time.perf_counter()
            TT.train(m, opt, loader, dev)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t) / len(src) * 1e3
        print(f"{kind:9s} {ms:.4f} ms per step ({TT.LAST_TRAIN_PATH})", flush=True)
        del m, opt
        harness._FAST.clear()
    _cache.prefetch = orig


if __name__ == "__main__":
    main()
