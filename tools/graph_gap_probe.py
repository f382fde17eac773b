"""What a hipGraph boundary costs on the GPU timeline: ms per iteration of
  A  graph replays back to back,
  B  an eager torch.randint before each replay (the fused training step's negatives draw),
  C  the same draw captured inside the graph (torch's graph-safe RNG: seed / offset kernels),
  D  two graphs back to back per iteration (a step split in two),
  E  the eager draw issued on a second stream, joined by an event before the replay,
for a graph of K tiny kernels. python tools/graph_gap_probe.py [--kernels 8] [--iters 400]"""
import argparse

import torch


def timed(fn, iters):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernels", type=int, default=8)
    ap.add_argument("--iters", type=int, default=400)
    args = ap.parse_args()
    dev = torch.device("cuda")
    x = torch.zeros(4096, device=dev)
    neg = torch.zeros(10000, dtype=torch.int64, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())

    def body():
        for _ in range(args.kernels):
            x.add_(1.0)

    body()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2):
        body()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        torch.randint(0, 59047, (10000,), device=dev, out=neg)
        body()
    side = torch.cuda.Stream()
    ev = torch.cuda.Event()

    def e_side():
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            torch.randint(0, 59047, (10000,), device=dev, out=neg)
            ev.record(side)
        torch.cuda.current_stream().wait_event(ev)
        g.replay()

    res = {
        "A replay": timed(g.replay, args.iters),
        "B eager draw + replay": timed(lambda: (torch.randint(0, 59047, (10000,), device=dev, out=neg), g.replay()),
                                       args.iters),
        "C captured draw": timed(gr.replay, args.iters),
        "D two graphs": timed(lambda: (g.replay(), g2.replay()), args.iters),
        "E side-stream draw + replay": timed(e_side, args.iters),
        "eager body": timed(body, args.iters),
        "eager draw": timed(lambda: torch.randint(0, 59047, (10000,), device=dev, out=neg), args.iters),
    }
    for k, v in res.items():
        print(f"{k:32s} {v:8.2f} us per iteration ({args.kernels} kernels per graph)", flush=True)


if __name__ == "__main__":
    main()
