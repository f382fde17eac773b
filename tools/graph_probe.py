"""Probe: the C2 K=3 forward replayed from a hipGraph vs issued eagerly."""
import os, sys, time
import torch
ROOT = "/root/repo" if os.path.exists("/root/repo") else os.getcwd()
sys.path.insert(0, os.path.join(ROOT, "movie-recommender-system-with-gnns_amd"))
import lgcn_amd
from lgcn_amd import synth
from lgcn_amd.plan import PropagationPlan

dev = torch.device("cuda")
g = synth.ml25m_shaped(seed=0)
ei = torch.from_numpy(g.edge_index).to(dev)
gen = torch.Generator(device=dev).manual_seed(0)
uw = torch.randn(g.num_users, 64, device=dev, generator=gen) * 0.01
iw = torch.randn(g.num_items, 64, device=dev, generator=gen) * 0.01
plan = PropagationPlan(ei, g.num_nodes, 256, side_split=g.num_users)
ref = lgcn_amd.propagate_forward(uw, iw, plan, 3)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        lgcn_amd.propagate_forward(uw, iw, plan, 3)
torch.cuda.current_stream().wait_stream(s)
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    out = lgcn_amd.propagate_forward(uw, iw, plan, 3)
graph.replay(); torch.cuda.synchronize()
print("graph bitwise eager:", bool(torch.equal(out, ref)), flush=True)
def t(fn, n=50, rounds=7):
    res = []
    for _ in range(rounds):
        torch.cuda.synchronize(); a = time.perf_counter()
        for _ in range(n): fn()
        torch.cuda.synchronize(); res.append((time.perf_counter() - a) / n * 1e3)
    return sorted(res)[rounds // 2]
for _ in range(2):
    print(f"eager {t(lambda: lgcn_amd.propagate_forward(uw, iw, plan, 3)):.4f} ms  graph {t(graph.replay):.4f} ms", flush=True)
