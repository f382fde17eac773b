"""Probe: can RCCL (torch.distributed "nccl") run W ranks that share the one GPU of a gpurun box?
Each rank runs the collectives the multi-GPU paths use (all_reduce, all_gather_into_tensor,
reduce_scatter_tensor, all_to_all_single, batch_isend_irecv) and checks the results.
python tools/rccl_probe.py [--world 2]  (spawns its own ranks; prints one line per rank)"""
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
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev,
                            timeout=datetime.timedelta(seconds=60))
    ok = []
    t = torch.full((8,), float(rank + 1), device=dev)
    dist.all_reduce(t)
    ok.append(("all_reduce", bool((t == world * (world + 1) / 2).all())))
    src = torch.arange(4, device=dev, dtype=torch.float32) + 10 * rank
    out = torch.empty(4 * world, device=dev)
    dist.all_gather_into_tensor(out, src)
    want = torch.cat([torch.arange(4, device=dev, dtype=torch.float32) + 10 * r for r in range(world)])
    ok.append(("all_gather_into_tensor", bool(torch.equal(out, want))))
    big = torch.arange(4 * world, device=dev, dtype=torch.float32) * (rank + 1)
    sh = torch.empty(4, device=dev)
    dist.reduce_scatter_tensor(sh, big)
    ok.append(("reduce_scatter_tensor",
               bool(torch.equal(sh, torch.arange(4 * rank, 4 * rank + 4, device=dev, dtype=torch.float32)
                                * (world * (world + 1) / 2)))))
    a2a_in = torch.arange(world * 2, device=dev, dtype=torch.float32) + 100 * rank
    a2a_out = torch.empty_like(a2a_in)
    dist.all_to_all_single(a2a_out, a2a_in)
    want = torch.cat([torch.arange(2 * rank, 2 * rank + 2, device=dev, dtype=torch.float32) + 100 * r
                      for r in range(world)])
    ok.append(("all_to_all_single", bool(torch.equal(a2a_out, want))))
    nxt, prv = (rank + 1) % world, (rank - 1) % world
    sbuf = torch.full((16,), float(rank), device=dev)
    rbuf = torch.empty(16, device=dev)
    reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend, sbuf, nxt), dist.P2POp(dist.irecv, rbuf, prv)])
    for r in reqs:
        r.wait()
    ok.append(("batch_isend_irecv", bool((rbuf == prv).all())))
    torch.cuda.synchronize()
    dist.barrier()
    print(f"rank {rank}: " + ", ".join(f"{n} {'ok' if v else 'WRONG'}" for n, v in ok), flush=True)
    dist.destroy_process_group()
    return 0 if all(v for _, v in ok) else 1


def main():
    if "RANK" in os.environ:
        sys.exit(rank_main())
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    args = ap.parse_args()
    port = free_port()
    procs = []
    for r in range(args.world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)], env=env))
    rcs = [p.wait() for p in procs]
    print(f"rccl_probe world {args.world}: exit codes {rcs}", flush=True)
    sys.exit(max(abs(c) for c in rcs))


if __name__ == "__main__":
    main()
