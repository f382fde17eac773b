"""Probe: can RCCL (torch.distributed "nccl") run W ranks that share the one GPU of a gpurun box,
and which of the collectives the multi-GPU paths use does gloo run on CUDA tensors? Each rank runs
all_reduce, all_gather_into_tensor (in place: the input a view of the output, as BlockExchange),
reduce_scatter_tensor, all_to_all_single and batch_isend_irecv on CUDA tensors, issued on a side
stream the compute stream then waits on (the nccl branches' pattern), and checks the results.
python tools/rccl_probe.py [--world 2] [--backend nccl|gloo]  (spawns its own ranks)"""
import argparse
import os
import socket
import subprocess
import sys


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def rank_main():
    import datetime

    import torch
    import torch.distributed as dist

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    backend = os.environ.get("PROBE_BACKEND", "nccl")
    kw = {"device_id": dev} if backend == "nccl" else {}
    dist.init_process_group(backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60), **kw)
    side = torch.cuda.Stream(dev)
    ok = []

    def on_side(name, fn, check):
        """fn issued on the side stream after an event on the compute stream, the compute stream
        waiting on the side stream's event before check() reads the result"""
        try:
            ready = torch.cuda.Event()
            ready.record(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                side.wait_event(ready)
                fn()
                done = torch.cuda.Event()
                done.record(side)
            torch.cuda.current_stream(dev).wait_event(done)
            ok.append((name, "ok" if check() else "WRONG"))
        except Exception as e:  # noqa: BLE001 — a probe: report and go on
            ok.append((name, f"raised {type(e).__name__}: {str(e).splitlines()[0][:120]}"))

    t = torch.full((8,), float(rank + 1), device=dev)
    on_side("all_reduce", lambda: dist.all_reduce(t), lambda: bool((t == world * (world + 1) / 2).all()))
    out = torch.zeros(4 * world, device=dev)
    out[4 * rank:4 * rank + 4] = torch.arange(4, device=dev, dtype=torch.float32) + 10 * rank
    want = torch.cat([torch.arange(4, device=dev, dtype=torch.float32) + 10 * r for r in range(world)])
    on_side("all_gather_into_tensor (in place)", lambda: dist.all_gather_into_tensor(out, out[4 * rank:4 * rank + 4]),
            lambda: bool(torch.equal(out, want)))
    big = torch.arange(4 * world, device=dev, dtype=torch.float32) * (rank + 1)
    sh = torch.empty(4, device=dev)
    on_side("reduce_scatter_tensor", lambda: dist.reduce_scatter_tensor(sh, big),
            lambda: bool(torch.equal(sh, torch.arange(4 * rank, 4 * rank + 4, device=dev, dtype=torch.float32)
                                     * (world * (world + 1) / 2))))
    a2a_in = torch.arange(world * 2, device=dev, dtype=torch.float32) + 100 * rank
    a2a_out = torch.empty_like(a2a_in)
    want2 = torch.cat([torch.arange(2 * rank, 2 * rank + 2, device=dev, dtype=torch.float32) + 100 * r
                       for r in range(world)])
    on_side("all_to_all_single", lambda: dist.all_to_all_single(a2a_out, a2a_in),
            lambda: bool(torch.equal(a2a_out, want2)))
    nxt, prv = (rank + 1) % world, (rank - 1) % world
    sbuf = torch.full((16,), float(rank), device=dev)
    rbuf = torch.empty(16, device=dev)

    def p2p():
        for r in dist.batch_isend_irecv([dist.P2POp(dist.isend, sbuf, nxt), dist.P2POp(dist.irecv, rbuf, prv)]):
            r.wait()

    on_side("batch_isend_irecv", p2p, lambda: bool((rbuf == prv).all()))
    torch.cuda.synchronize()
    dist.barrier()
    print(f"rank {rank} ({backend}): " + "; ".join(f"{n} {v}" for n, v in ok), flush=True)
    dist.destroy_process_group()
    return 0 if all(v == "ok" for _, v in ok) else 1


def main():
    if "RANK" in os.environ:
        sys.exit(rank_main())
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    args = ap.parse_args()
    port = free_port()
    procs = []
    for r in range(args.world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PROBE_BACKEND=args.backend)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)], env=env))
    rcs = [p.wait() for p in procs]
    print(f"rccl_probe world {args.world} {args.backend}: exit codes {rcs}", flush=True)
    sys.exit(max(abs(c) for c in rcs))


if __name__ == "__main__":
    main()
