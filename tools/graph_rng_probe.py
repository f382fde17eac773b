"""Probe: does torch.cuda.CUDAGraph.replay() launch the RNG seed/offset fills when the captured
graph holds no RNG op? Replays a graph without and one with torch.randint, 20 times each, marked
by distinct kernels, for rocprofv3 --kernel-trace to count the fills between them."""
import torch

dev = torch.device("cuda")
x = torch.zeros(1024, device=dev)
y = torch.empty(1024, dtype=torch.int64, device=dev)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(2):
        x.mul_(1.0)
        torch.randint(0, 100, (1024,), device=dev, out=y)
torch.cuda.current_stream().wait_stream(s)
g_plain = torch.cuda.CUDAGraph()
with torch.cuda.graph(g_plain):
    x.mul_(1.0)
g_rng = torch.cuda.CUDAGraph()
with torch.cuda.graph(g_rng):
    torch.randint(0, 100, (1024,), device=dev, out=y)
torch.cuda.synchronize()
for _ in range(20):
    g_plain.replay()
torch.cuda.synchronize()
x.sub_(0.0)  # marker between the two phases
torch.cuda.synchronize()
for _ in range(20):
    g_rng.replay()
torch.cuda.synchronize()
print("done")
