"""Headline benchmark: edges propagated/s of K-layer LightGCN propagation (BASELINE.json metric).

Workload (BASELINE.json configs[1]): MovieLens-25M-shaped full bipartite graph
(U=162,541, I=59,047, 12.45M unique rating>=4 pairs -> E = 24.9M directed edges), K=3, d=64,
fp32. One step = one full K-layer forward propagation (LightGCN.forward semantics, reference
models/light_gcn.py:28-40) with the plan (CSR + gcn_norm + schedule) already built and the
embedding tables resident in HBM. value = K * E / wall time per step: ONE graph at every N.

Multi-GPU: `python bench.py --gpus N` starts N rank processes itself (one per GPU; under
torchrun, which sets WORLD_SIZE, it is one of them). Strong scaling. C2 is sharded over an R x F
grid (lgcn_amd.sharded): F column groups (each propagates d/F columns, no exchange between them)
times R row groups, in one of three exchange modes timed per grid: allgather / p2p (each rank
propagates its own edge-balanced destination rows of the same graph, and each layer's two output
blocks (user rows, item rows) are all-gathered, or sent peer to peer, over RCCL within the column
group on a side stream while the other half-layer computes) and reduce (users sharded, every rank
sums its users' share of every item row; the item partials are all-reduced per layer, the last
layer reduce-scattered). With R = 1 a rank's columns are bitwise the 1-GPU result; with R > 1
ranks run the plain schedule at chunk 128, whose rows are within 1e-5 of the sliced 1-GPU result
(allgather / p2p: bitwise the 1-GPU plain schedule at that chunk; reduce: an item row is the sum
of R partial chains).
C5 (--config c5) is feature-sharded: d/N columns per rank, no collective. The barrier and the
max-over-ranks time go over RCCL.

Also reported (one JSON line on rank 0):
  roofline     — the dominant kernel (the item pass, k_spmm_vec; at C2 one launch per source
                 slice, lgcn_amd.sliced), its launch time measured live with HIP events on its
                 launching stream. achieved = memory-side bytes per launch (rocprofv3 FETCH_SIZE
                 x calibration + WRITE_SIZE, profiles/pmc_traffic.json, measured on this workload)
                 / launch time, frac = achieved / 8 TB/s; without a PMC entry the compulsory bytes
                 of the schedule stand in (basis "compulsory", a lower bound). Also: the schedule's
                 compulsory bytes, SURVEY §8d's no-reuse algorithmic bytes as effective_GBps.
  cpu_baseline — the reference's CPU op sequence (PyG 2.4.0 LGConv restated with torch CPU
                 primitives, oracle/lgconv_torch.py) on the whole C2 graph, rank 0, N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "movie-recommender-system-with-gnns_amd"))
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)
GATHER_L2_PEAK_GBS = 18800.0  # fully L2-resident row gathers, chip-wide (MI355X_MICROARCH.md, upper end)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


TIMER_EVERY = 5


class LaunchTimer:
    """HIP-event brackets around the dominant kernel's launches, on the launching stream; each
    bracket covers n item-pass launches (a layer's source slices)."""

    def __init__(self):
        import torch

        self.torch = torch
        self.pairs = []
        self.active = False

    def __call__(self, d, n=1):
        timer = self

        class _Ctx:
            def __enter__(self_):
                if timer.active:
                    s = timer.torch.cuda.Event(enable_timing=True)
                    s.record(timer.torch.cuda.current_stream())
                    self_.s = s

            def __exit__(self_, *exc):
                if timer.active:
                    e = timer.torch.cuda.Event(enable_timing=True)
                    e.record(timer.torch.cuda.current_stream())
                    timer.pairs.append((self_.s, e, n))
                return False

        return _Ctx()

    def mean_ms(self):
        """Average time of one launch (brackets include the ~1.5 us gaps between a layer's slices)."""
        if not self.pairs:
            return None
        return sum(s.elapsed_time(e) for s, e, _ in self.pairs) / sum(n for _, _, n in self.pairs)


def kernel_source_sha16() -> str:
    """sha256 prefix of the dominant kernel's source (csrc/lgcn_spmm.hip + the shared header)."""
    import hashlib

    h = hashlib.sha256()
    for f in ("lgcn_spmm.hip", "lgcn_common.h"):
        h.update((ROOT / "movie-recommender-system-with-gnns_amd" / "csrc" / f).read_bytes())
    return h.hexdigest()[:16]


def traffic_signature(workload: str, kernel: str, launches: int, n_items: int, edges: int, graph: dict) -> dict:
    """What a PMC traffic entry was measured on: the workload, the kernel instance, the launch
    schedule (launches per layer, items and edges of one layer's item pass), the graph's degree
    statistics and the kernel source. A committed entry counts only when every field matches."""
    return {"workload": workload, "kernel": kernel, "launches_per_layer": int(launches),
            "items_per_layer": int(n_items), "edges_per_layer": int(edges), "graph": graph,
            "kernel_source_sha16": kernel_source_sha16()}


def load_traffic(signature: dict):
    """(memory-side bytes per launch of the dominant kernel from the committed PMC profile, or None;
    why not) — None unless the entry's recorded signature equals this run's."""
    p = ROOT / "profiles" / "pmc_traffic.json"
    if not p.exists():
        return None, "no profiles/pmc_traffic.json"
    try:
        ent = json.loads(p.read_text()).get(signature["workload"])
    except (OSError, ValueError) as e:
        return None, f"unreadable pmc_traffic.json: {e}"
    if ent is None:
        return None, "no PMC entry for this workload"
    rec = ent.get("signature")
    if rec != signature:
        diff = sorted(k for k in set(signature) | set(rec or {}) if (rec or {}).get(k) != signature.get(k))
        return None, f"PMC entry measured on another plan/kernel (differs in: {', '.join(diff)})"
    return ent.get("hbm_bytes_per_launch"), None


def kernel_lpr(d):
    """Template of the item-pass instance lgcn_spmm launches for width d (csrc/lgcn_spmm.hip)."""
    return {4: "1,1,8", 8: "2,1,8", 16: "4,1,8", 32: "8,1,8", 64: "16,1,8", 128: "32,1,8", 256: "64,1,8",
            512: "64,2,4", 1024: "64,4,2"}.get(d, "scalar")


def init_dist(backend, dev):
    import datetime

    import torch.distributed as dist

    # a bounded timeout: a rank stuck in a collective ends the run instead of holding the node
    timeout = datetime.timedelta(seconds=int(os.environ.get("LGCN_DIST_TIMEOUT_S", "300")))
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev, timeout=timeout)
    else:
        dist.init_process_group(backend, timeout=timeout)


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def child_envs(n: int, port: int, base=None) -> list:
    """The environment of each of n rank processes (what torch.distributed.run would set):
    RANK = LOCAL_RANK = i, WORLD_SIZE = LOCAL_WORLD_SIZE = n, rendezvous on 127.0.0.1:port."""
    base = dict(os.environ if base is None else base)
    envs = []
    for i in range(n):
        e = dict(base)
        e.update(RANK=str(i), LOCAL_RANK=str(i), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        envs.append(e)
    return envs


def launch_ranks(n: int, argv: list, script=None, relayed: list | None = None) -> int:
    """`python bench.py --gpus N` outside torchrun: start N rank processes of this script (one per
    GPU, LOCAL_RANK = GPU index) and wait for them. This process touches no GPU (it imports neither
    torch nor lgcn_amd). Rank 0's stdout (the JSON line) is relayed; if any rank fails the others
    are stopped and its exit code is returned. script: the rank program (tests; default this file);
    relayed: a list that receives the relayed JSON lines."""
    import signal
    import subprocess

    port = free_port()
    cmd = [sys.executable, "-u", str(script or pathlib.Path(__file__).resolve()), *argv]
    log(f"launch: {n} rank processes on 127.0.0.1:{port}: {' '.join(cmd[2:])}")

    def die_with_parent():
        # a rank gets SIGTERM if this launcher dies (even by SIGKILL): no orphan holds a GPU
        import ctypes

        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, int(signal.SIGTERM))  # PR_SET_PDEATHSIG

    procs = [subprocess.Popen(cmd, env=e, stdout=subprocess.PIPE if i == 0 else subprocess.DEVNULL,
                              start_new_session=True, preexec_fn=die_with_parent)
             for i, e in enumerate(child_envs(n, port))]

    def stop_all(signum, frame):
        # the launcher was told to stop (a driver timeout): stop every rank's process group, then go
        for q in procs:
            try:
                os.killpg(q.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
        deadline = time.monotonic() + 20
        for q in procs:
            try:
                q.wait(timeout=max(0.1, deadline - time.monotonic()))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(q.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
        sys.exit(128 + signum)

    for sig in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP):
        signal.signal(sig, stop_all)
    import threading

    out = relayed if relayed is not None else []

    def relay():
        # the JSON line to stdout; anything else a library prints there (gloo, RCCL) to stderr
        for line in procs[0].stdout:
            if line.lstrip().startswith(b"{"):
                out.append(line)
                sys.stdout.buffer.write(line)
                sys.stdout.flush()
            else:
                sys.stderr.buffer.write(line)
                sys.stderr.flush()

    t = threading.Thread(target=relay, daemon=True)
    t.start()
    rc, stop_at = 0, None
    pending = set(range(n))
    while pending:
        for i in sorted(pending):
            r = procs[i].poll()
            if r is None:
                continue
            pending.discard(i)
            if r != 0 and rc == 0:
                rc = r if r > 0 else 128 - r
                stop_at = time.monotonic()
                log(f"launch: rank {i} exited with {r}; stopping the other ranks")
                for j in pending:
                    try:
                        os.killpg(procs[j].pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
        if stop_at is not None and pending and time.monotonic() - stop_at > 30:
            for j in pending:  # ranks that ignore SIGTERM (stuck in a collective)
                try:
                    os.killpg(procs[j].pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
            stop_at = time.monotonic()
        time.sleep(0.2)
    t.join(timeout=10)
    if rc == 0 and not out:
        log("launch: rank 0 printed nothing")
        rc = 1
    return rc


def launch_with_fallback(args, launch=None) -> int:
    """launch_ranks, and once more without the peer-send grid candidates (LGCN_GRID_NO_P2P=1) when
    a C2 grid run ended with no result: those candidates are timed last and are the one exchange
    outside RCCL's plain collectives, so a rank stuck in one ends the run at the process-group
    timeout before a grid is picked — the second launch then times the plain candidates only."""
    launch = launch or launch_ranks
    out = []
    rc = launch(args.gpus, sys.argv[1:], relayed=out)
    if (rc != 0 and not out and args.gpus >= 3 and args.workload == "propagate" and args.config == "c2"
            and not args.shard and os.environ.get("LGCN_GRID_NO_P2P") != "1"):
        log(f"launch: no result (exit {rc}); launching again without the peer-send grid candidates")
        os.environ["LGCN_GRID_NO_P2P"] = "1"
        rc = launch(args.gpus, sys.argv[1:], relayed=out)
    return rc


def parse_tune(items) -> dict:
    """--tune FIELD=VALUE ... -> {field: value} typed by lgcn_amd.tuning.Tuning (checked here, set by
    apply_tune in each rank process)."""
    import dataclasses

    out = {}
    if not items:
        return out
    sys.path.insert(0, str(ROOT / "movie-recommender-system-with-gnns_amd"))
    from lgcn_amd.tuning import Tuning

    types = {f.name: str(f.type) for f in dataclasses.fields(Tuning)}
    for it in items:
        k, _, v = it.partition("=")
        if k not in types:
            raise SystemExit(f"--tune: unknown field {k!r} (fields: {', '.join(types)})")
        t = types[k]
        if v == "None" and "None" in t:
            out[k] = None
            continue
        out[k] = (v not in ("0", "false", "False") if "bool" in t else
                  float(v) if "float" in t else int(v) if "int" in t else v)
    return out


def _batch_chunk_for(edges: int) -> int:
    from lgcn_amd.train_step import batch_chunk_for

    return batch_chunk_for(edges)


def apply_tune(tuned: dict) -> None:
    if tuned:
        from lgcn_amd import tuning

        tuning.set_tuning(**tuned)
        log(f"tuning: {tuned}")


def cpu_share():
    """(CPUs in this process's affinity mask, cgroup CPU quota or None, physical cores of the machine)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    phys = None
    try:
        import psutil

        phys = psutil.cpu_count(logical=False)
    except Exception:
        pass
    return aff, quota, phys


def cpu_baseline(graph, K, d, seconds_budget=20.0, label="C2"):
    """Reference CPU path (torch primitives of PyG 2.4.0 LGConv, oracle/lgconv_torch.py) on the
    WHOLE C2 edge set, with every CPU of the affinity mask; when a cgroup quota
    caps the process below that, the quota's thread count is timed too and the faster is kept."""
    import torch

    from oracle.lgconv_torch import time_csr_forward, time_reference_forward

    aff, quota, phys = cpu_share()
    counts = [aff] + ([quota] if quota and quota < aff else [])
    ei = torch.from_numpy(graph.edge_index)
    g = torch.Generator().manual_seed(0)
    uw = torch.randn(graph.num_users, d, generator=g) * 0.01
    iw = torch.randn(graph.num_items, d, generator=g) * 0.01
    runs, cold = {}, {}
    for threads in counts:  # per thread count: a cold run (warm-up), then a warm run picks the count
        torch.set_num_threads(threads)
        t0 = time.perf_counter()
        cold[threads] = time_reference_forward(uw, iw, ei, K, reps=1, warmup=False)
        log(f"cpu_baseline: all {ei.shape[1]} edges, {threads} threads, {cold[threads]:.3f} s/forward (cold) "
            f"({time.perf_counter() - t0:.1f} s total)")
    best_cold = min(cold.values())
    for threads in counts:
        if cold[threads] > 2 * best_cold:  # cannot plausibly win: not worth a warm run
            runs[threads] = (cold[threads], 1)
            continue
        torch.set_num_threads(threads)
        t = time_reference_forward(uw, iw, ei, K, reps=1, warmup=False)
        runs[threads] = (t, 1)
        log(f"cpu_baseline: {threads} threads, {t:.3f} s/forward (warm)")
    threads = min(runs, key=lambda k: runs[k][0])
    torch.set_num_threads(threads)
    # the chosen count: the median of 3 more warm runs
    reps = 3
    t0 = time.perf_counter()
    t = time_reference_forward(uw, iw, ei, K, reps=reps, warmup=False)
    runs[threads] = (t, reps)
    log(f"cpu_baseline: {threads} threads, median of {reps}: {t:.3f} s/forward ({time.perf_counter() - t0:.1f} s)")
    t1 = time.perf_counter()
    tc = time_csr_forward(uw, iw, ei, K, reps=3)
    log(f"cpu_baseline csr: {ei.shape[1]} edges, {threads} threads, {tc:.3f} s/forward "
        f"({time.perf_counter() - t1:.1f} s total)")
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            model = next(line.split(":", 1)[1].strip() for line in f if line.startswith("model name"))
    except (OSError, StopIteration):
        pass
    return {"value": K * ei.shape[1] / t, "unit": "edges/s", "cores": threads, "kind": "port", "cpu_model": model,
            "affinity_cpus": aff, "cgroup_cpu_quota": quota, "physical_cores_machine": phys,
            "threads_timed": {str(k): K * ei.shape[1] / v[0] for k, v in runs.items()},
            "csr_spmm": {"value": K * ei.shape[1] / tc, "unit": "edges/s", "cores": threads,
                         "sample": f"all {ei.shape[1]} {label} edges, K={K} d={d}: gcn_norm-weighted CSR built once, "
                                   f"torch.sparse.mm per layer + layer mean, median of 3"},
            "sample": f"all {ei.shape[1]} {label} edges (no sampling), all {graph.num_nodes} nodes, K={K} d={d} forward: "
                      f"index_select -> mul -> scatter_add_ with gcn_norm per layer (PyG 2.4.0 LGConv op sequence, "
                      f"torch {torch.__version__} CPU), thread count picked by a warm run after a cold one, then the "
                      f"median of {reps}"}


SETTLE_GROUP = 5        # warm-up steps per settle check
SETTLE_TOL = 0.005      # settled: a group's mean step is no more than 0.5 % faster than the group before
SETTLE_MAX_S = 1.0      # at most this much extra warm-up (seconds of wall time)


def settle_warmup(step, torch, dist=None, dev=None) -> dict:
    """Untimed warm-up beyond --warmup until the step time stops falling. On a fresh box the first
    ~25 ms of back-to-back steps run up to 14 % slower than the steady state (a clock ramp:
    profiles/r05a_settle/, per-step series at 20/5, 50/10 and 200/5), so W = 5 warm-up steps alone
    leave the driver's 20 timed steps ~3 % slow. Steps run in groups of SETTLE_GROUP, each group
    bracketed by HIP events on the current stream; warm-up ends at the first group whose mean is
    within SETTLE_TOL of the previous group's (every rank agrees: the max over ranks of the
    continue flag), or after SETTLE_MAX_S. The timed region is untouched: all K timed steps' work
    stays inside it."""
    groups, prev = [], None
    t_end = time.perf_counter() + SETTLE_MAX_S
    while True:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(torch.cuda.current_stream())
        for _ in range(SETTLE_GROUP):
            step()
        b.record(torch.cuda.current_stream())
        b.synchronize()
        ms = a.elapsed_time(b) / SETTLE_GROUP
        groups.append(round(ms, 5))
        more = float(prev is None or ms < prev * (1 - SETTLE_TOL))
        late = float(time.perf_counter() >= t_end)
        if dist is not None:
            flag = torch.tensor([more, late], dtype=torch.float64, device=dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MAX)
            more, late = float(flag[0].item()), float(flag[1].item())
        if not more or late:
            return {"steps": SETTLE_GROUP * len(groups), "group_mean_ms": groups}
        prev = ms


def collective_fn(dist, torch, op: str, nbytes: int, group, n: int, dev):
    """(fn, buffer bytes): one `op` over `group` (n ranks) of about nbytes (the whole buffer: the
    all_reduce's tensor, reduce_scatter's / all_to_all's input, all_gather's output), fp32."""
    m = max(1, -(-int(nbytes) // (4 * n)))  # floats per rank slice
    f = dict(dtype=torch.float32, device=dev)
    if op == "all_reduce":
        buf = torch.zeros(n * m, **f)
        return (lambda: dist.all_reduce(buf, group=group)), 4 * n * m
    if op == "reduce_scatter":
        inp, out = torch.zeros(n * m, **f), torch.empty(m, **f)
        return (lambda: dist.reduce_scatter_tensor(out, inp, group=group)), 4 * n * m
    if op == "all_gather":
        inp, out = torch.zeros(m, **f), torch.empty(n * m, **f)
        return (lambda: dist.all_gather_into_tensor(out, inp, group=group)), 4 * n * m
    if op == "all_to_all":
        inp, out = torch.zeros(n * m, **f), torch.empty(n * m, **f)
        return (lambda: dist.all_to_all_single(out, inp, group=group)), 4 * n * m
    raise ValueError(f"unknown collective {op!r}")


def probe_collectives(dist, torch, dev, specs, reps: int = 10, sync=None) -> list:
    """Untimed by the bench line: each spec {name, op, bytes, group, ranks} — a collective the
    multi-GPU step or its projection (tools/project_scale.py, tools/project_c4.py) prices — run
    2 + reps times on this node's ranks (all column groups at once, as in the step); ms is the
    mean per call, the max over ranks; bus bandwidth by the rccl-tests convention
    (tools/scale_model.BUS_FACTOR). A collective that raises on any rank is recorded as failed on
    every rank (one all_reduce of [ms, failed] per spec)."""
    from tools.scale_model import bus_gbps

    sync = sync or (lambda: torch.cuda.synchronize())
    out = []
    for sp in specs:
        rec = {"name": sp["name"], "op": sp["op"], "ranks": int(sp["ranks"]), "bytes": int(sp["bytes"])}
        ms, failed = 0.0, 0.0
        try:
            fn, rec["bytes"] = collective_fn(dist, torch, sp["op"], sp["bytes"], sp.get("group"), sp["ranks"], dev)
            for _ in range(2):
                fn()
            sync()
            dist.barrier()
            t = time.perf_counter()
            for _ in range(reps):
                fn()
            sync()
            ms = (time.perf_counter() - t) / reps * 1e3
        except Exception as e:  # noqa: BLE001 — recorded, agreed on
            failed = 1.0
            rec["error"] = f"{type(e).__name__}: {e}"[:160]
            sync()
        agree = torch.tensor([ms, failed], dtype=torch.float64, device=dev)
        dist.all_reduce(agree, op=dist.ReduceOp.MAX)
        ms, failed = float(agree[0].item()), bool(agree[1].item())
        if failed:
            rec.update(ms=None, busbw_GBps=None, algbw_GBps=None, failed=True)
        else:
            rec.update(ms=float(f"{ms:.5g}"), busbw_GBps=float(f"{bus_gbps(sp['op'], rec['bytes'], rec['ranks'], ms):.4g}"),
                       algbw_GBps=float(f"{rec['bytes'] / (ms * 1e-3) / 1e9:.4g}"))
        out.append(rec)
    return out


def project_chosen_grid(st, K: int, collectives: list, measured_ms: float, torch, dist) -> dict:
    """projected_ms_per_step of the chosen C2 grid beside the measured one: the rank's own pieces
    (partial pass, user pass, their pair launch; HIP events, untimed) and the collectives just
    timed on this node, through tools/scale_model.simulate (the model tools/project_scale.py
    prices with assumed bandwidths). The max over ranks of each piece."""
    mode = str(st.get("mode"))
    grid = st["grid"]
    if not mode.startswith("reduce"):
        return {"grid": f"{grid.R}x{grid.F}", "mode": st.get("mode"), "measured_ms_per_step": measured_ms,
                "projected_ms_per_step": None,
                "note": "no reduce exchange: the step is the rank's compute (its trial time)"}
    from tools.scale_model import simulate

    from lgcn_amd import _ffi

    rplan = st["splan"]
    x0u, x0i = st["x0"]
    d = x0u.shape[1]
    dev = x0u.device
    part = torch.zeros((rplan.I_pad, d), device=dev)
    acc = (torch.zeros((x0u.shape[0], d), device=dev), torch.zeros((x0i.shape[0], d), device=dev), x0u.shape[0])
    y = torch.empty((x0u.shape[0], d), device=dev)

    def timed(fn, reps=20):
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

    with torch.no_grad():
        t = torch.tensor([timed(lambda: rplan.run_partial(x0u, part)),
                          timed(lambda: rplan.run_users(x0i, None, acc, y, _ffi.EPI_ADD, 1.0, 1.0)),
                          timed(lambda: rplan.run_pair(x0u, part, x0i, None, acc, y, _ffi.EPI_ADD, 1.0, 1.0))],
                         dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    t_p, t_u, t_pair = (float(v) for v in t.tolist())
    by = {c["name"]: c for c in collectives}
    key = f"{grid.R}x{grid.F}_items_"
    if "a2a" in mode:  # all_to_all + ordered sums + all_gather; the last layer stops after the sums
        parts = [by.get(key + "all_to_all"), by.get(key + "all_gather")]
        t_ar = sum(c["ms"] for c in parts) if all(c and c["ms"] is not None for c in parts) else None
        t_rs = parts[0]["ms"] if parts[0] and parts[0]["ms"] is not None else None
    else:
        ar, rs = by.get(key + "all_reduce"), by.get(key + "reduce_scatter")
        t_ar = ar["ms"] if ar and ar["ms"] is not None else None
        t_rs = rs["ms"] if rs and rs["ms"] is not None else None
    out = {"grid": f"{grid.R}x{grid.F}", "mode": mode, "measured_ms_per_step": measured_ms,
           "pieces_ms": {"partial_pass": t_p, "user_pass": t_u, "pair": t_pair},
           "collective_ms": {"all_reduce_like": t_ar, "reduce_scatter_like": t_rs},
           "compute_alone_ms": K * ((t_pair) if mode.endswith("fused") else (t_p + t_u))}
    if t_ar is None or t_rs is None:
        out["projected_ms_per_step"] = None
        out["note"] = "a priced collective failed on this node"
        return out
    out["projected_ms_per_step"] = simulate(K, t_p, t_u, t_pair, t_ar, t_rs, mode.endswith("fused"))
    out["measured_over_projected"] = measured_ms / out["projected_ms_per_step"]
    return out


def c2_collective_specs(world: int, d_full: int, num_items: int, groups: dict, candidates) -> list:
    """The collectives the C2 reduce grids exchange (lgcn_amd.sharded.ItemReducer): per R > 1
    grid, its column group's item partial table (I x d/F fp32) all-reduced K-1 times and
    reduce-scattered once per step (ring), or all_to_all'd + all_gathered (a2a); and the
    latency of a tiny all_reduce in the group and in the world."""
    specs, seen = [], set()
    for R, F, mode in candidates:
        if R == 1 or (R, F) in seen or not str(mode).startswith("reduce"):
            continue
        seen.add((R, F))
        nb = num_items * (d_full // F) * 4
        g = groups.get((R, F))
        for op in ("all_reduce", "reduce_scatter", "all_to_all", "all_gather"):
            specs.append(dict(name=f"{R}x{F}_items_{op}", op=op, bytes=nb, group=g, ranks=R))
        specs.append(dict(name=f"{R}x{F}_latency_all_reduce_8B", op="all_reduce", bytes=8, group=g, ranks=R))
    specs.append(dict(name=f"world_latency_all_reduce_8B", op="all_reduce", bytes=8, group=None, ranks=world))
    return specs


def c4_collective_specs(world: int, dp_mode: str, exchange, cols, num_items: int, d: int, max_b: int) -> list:
    """The collectives a C4 training step exchanges in the chosen mode (tools/project_c4.py prices
    them): owner — the gradient blocks' and the replies' all_to_alls and the clip partials'
    all_gather; hybrid — the item gradient table's all_reduce and the users' record all_gather;
    replicated — the record blocks' all_gather; columns — the triplets' [B, 6] all_reduce. Plus a
    tiny all_reduce's latency."""
    specs = []
    if dp_mode == "owner" and exchange is not None:
        specs += [dict(name="owner_blocks_all_to_all", op="all_to_all", bytes=exchange.send.numel() * 4),
                  dict(name="owner_replies_all_to_all", op="all_to_all", bytes=exchange.reply_send.numel() * 4),
                  dict(name="owner_norm_all_gather", op="all_gather", bytes=exchange.partials_all.numel() * 4)]
    elif dp_mode == "hybrid" and exchange is not None:
        specs += [dict(name="hybrid_items_all_reduce", op="all_reduce", bytes=num_items * d * 4),
                  dict(name="hybrid_users_all_gather", op="all_gather", bytes=world * exchange.blk * 4)]
    elif exchange is not None:
        specs += [dict(name="records_all_gather", op="all_gather", bytes=world * exchange.blk * 4)]
    if cols is not None:
        specs += [dict(name="columns_bpr_sums_all_reduce", op="all_reduce", bytes=6 * max_b * 4)]
    specs.append(dict(name="world_latency_all_reduce_8B", op="all_reduce", bytes=8))
    for sp in specs:
        sp.update(group=None, ranks=world)
    return specs


def schedule_traffic(sched, n_src_rows: int, d: int):
    """(compulsory bytes of one middle layer's item pass over `sched`, its launches, edges, rows
    finished in the pass): every source
    row read once, each edge's int32 index + fp32 weight, each lgcn_item_t, the ADD epilogue of
    each row finished in the pass (y write + acc read + write), the running-sum read/write of each
    non-FIRST / non-LAST slice segment, and the hub rows' partial slots written."""
    import torch

    from lgcn_amd.sliced import ITEM_FIRST, ITEM_LAST, SlicedDirection

    row = 4 * d
    if isinstance(sched, SlicedDirection):
        n = sum(n for _, n in sched.launches)
        ld = sched.items[:n, 1].contiguous().view(torch.int32).view(-1, 2)
        ln, rowi = ld[:, 0], ld[:, 1] >= 0
        run_rw = int(((ln & ITEM_FIRST) == 0)[rowi].sum()) + int(((ln & ITEM_LAST) == 0)[rowi].sum())
        finished = int(((ln & ITEM_LAST) != 0)[rowi].sum())
        edges = int((ln & 0x1FFFFFFF).sum())
        launches = sched.n_launches
    else:
        n = sched.n_items
        ld = sched.items[:n, 1].contiguous().view(torch.int32).view(-1, 2)
        run_rw, finished, launches = 0, int((ld[:, 1] >= 0).sum()), 1
        edges = int(ld[:, 0].sum())
    per_layer = (n_src_rows * row + edges * 8 + n * 16 + finished * 3 * row + run_rw * row
                 + sched.n_partials * row)
    return per_layer, launches, edges, finished + sched.n_splits, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", choices=["c2", "c5"], default="c2",
                    help="propagate workload: c2 = ML-25M-shaped K=3 d=64 (headline); c5 = 10M x 1M x 5e8, K=4 d=256")
    ap.add_argument("--layers", type=int, default=None, help="K (default 3 for c2, 4 for c5)")
    ap.add_argument("--dim", type=int, default=None, help="d (default 64 for c2, 256 for c5; train: 128)")
    ap.add_argument("--scale", type=float, default=1.0, help="graph scale vs ML-25M (1.0 = C2)")
    ap.add_argument("--chunk", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--tune", action="append", default=[], metavar="FIELD=VALUE",
                    help="A/B: set one lgcn_amd.tuning field for the run (repeatable; the defaults are the "
                         "measured choices, and the JSON line lists any field set)")
    ap.add_argument("--step-times", action="store_true",
                    help="diagnostic: a HIP event at every timed step boundary; the per-step ms series goes "
                         "into the JSON line (step_ms) and to stderr")
    ap.add_argument("--shard", default=None,
                    help="c2, N > 1: RxF grid (R row groups x F column groups, R*F = N); default: every "
                         "lgcn_amd.sharded.grid_candidates grid is timed for a few steps and the fastest runs")
    ap.add_argument("--exchange-mode", choices=["allgather", "p2p", "reduce", "reduce-fused", "reduce-a2a",
                                                "reduce-a2a-fused"], default="allgather",
                    help="c2 with --shard and R > 1: one all_gather per block, or sends to every peer")
    ap.add_argument("--workload", choices=["propagate", "train"], default="propagate",
                    help="propagate: C2 headline (default); train: C3/C4 Cluster-GCN training steps")
    ap.add_argument("--parts", type=int, default=1024, help="train: Cluster-GCN parts")
    ap.add_argument("--graph", choices=["ml25m", "planted"], default="ml25m",
                    help="train: the ML-25M-shaped random graph (f_intra ~3%%, ~20k-edge batches) or the "
                         "ML-25M-sized planted-community graph (f_intra ~46%%, ~324k-edge batches)")
    ap.add_argument("--parts-per-batch", type=int, default=32, help="train: parts per step")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) for runs; gloo to rehearse N ranks on one GPU")
    ap.add_argument("--torch-adam", action="store_true", help="train: torch Adam + clip_grad_norm_ (reference ops)")
    ap.add_argument("--no-graphs", action="store_true", help="train: run the fused step eagerly (no hipGraph replay)")
    ap.add_argument("--exchange", action="store_true",
                    help="train, N=1: run the row exchange anyway (measures its kernels; N>1 always uses it)")
    ap.add_argument("--dp-lr", choices=["sqrt", "same"], default="sqrt",
                    help="train, data parallel: Adam lr 1e-3 * sqrt(W) (default; lgcn_amd.distributed.dp_lr) or 1e-3")
    ap.add_argument("--dp-mode", choices=["auto", "replicated", "owner", "columns", "hybrid"], default="auto",
                    help="train, N > 1: column-sharded exact training (every rank the same batches on d/N "
                         "columns, one [B, 6] all_reduce per step — the one-GPU step's semantics, so Recall is "
                         "the one-GPU run's), or data parallel over disjoint parts with a replicated row-lazy "
                         "Adam (all_gather of every rank's gradient rows) or an owner-sharded one (two "
                         "all_to_alls) — W-times fewer, larger Adam steps: Recall@20 within the +-0.002 band "
                         "with little margin at W = 8, Recall@100 outside it (tests/test_gpu_dp_recall.py). "
                         "auto: the projection's pick (tools/project_c4.py, DESIGN §7): columns at N <= 2, "
                         "owner from N = 4")
    ap.add_argument("--no-harness", action="store_true",
                    help="train, N=1: skip timing utils.train_test.train() both ways after the bench line's run")
    ap.add_argument("--dense-adam", action="store_true",
                    help="train: dense FusedAdam over all rows every step instead of the row-lazy exact Adam")
    ap.add_argument("--autograd", action="store_true",
                    help="train: reference-style step (compute_embeddings + bpr_loss + autograd) instead of "
                         "the fused no-autograd step")
    args = ap.parse_args()
    args.tuned = parse_tune(args.tune)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # plain `python bench.py --gpus N`: become the launcher of N ranks (torchrun sets WORLD_SIZE)
        sys.exit(launch_with_fallback(args))
    if args.workload == "train":
        return run_train(args)

    import numpy as np
    import torch
    import torch.distributed as dist

    import lgcn_amd
    from lgcn_amd import synth
    from lgcn_amd.plan import DEFAULT_CHUNK, PropagationPlan, sliced_chunk
    from lgcn_amd.sliced import SlicedDirection

    apply_tune(args.tuned)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    dev = torch.device("cuda", local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    distributed = world > 1
    if distributed:
        init_dist(args.dist_backend, dev)

    c5 = args.config == "c5"
    K = args.layers if args.layers is not None else (4 if c5 else 3)
    d = args.dim if args.dim is not None else (256 if c5 else 64)
    d_full = d
    chunk = args.chunk or DEFAULT_CHUNK
    t0 = time.perf_counter()
    graph = None
    sharded = not c5 and distributed
    if c5:
        # C5: one synthetic 10M x 1M x 5e8-edge graph (same seed on every rank, generated on the GPU).
        # N > 1 ranks shard the embedding COLUMNS (feature-sharded propagation): every
        # rank runs the full plan on d/W columns, no collective; value = K*E / time (strong scaling).
        s = args.scale
        U, I = int(synth.C5_USERS * s), int(synth.C5_ITEMS * s)
        ei = synth.bipartite_device(U, I, int(synth.C5_PAIRS * s), seed=0, device=dev)
        if d % world or (d // world) % 4:
            raise SystemExit(f"c5 feature sharding needs d % (4*W) == 0 (d={d}, W={world})")
        d = d // world
        N, E = U + I, int(ei.shape[1])
        log(f"[rank {rank}] c5 graph U={U} I={I} E={E} on device, d={d_full} -> {d} columns per rank "
            f"({time.perf_counter() - t0:.1f} s)")
    else:
        # C2: ONE graph (seed 0 on every rank); N > 1 ranks split its destination rows
        graph = synth.ml25m_shaped(seed=0, scale=args.scale)
        log(f"[rank {rank}] graph U={graph.num_users} I={graph.num_items} E={graph.num_edges} "
            f"{graph.degree_stats()} ({time.perf_counter() - t0:.1f} s)")
        U, I, N, E = graph.num_users, graph.num_items, graph.num_nodes, graph.num_edges
        ei = torch.from_numpy(graph.edge_index).to(dev)
    # the model's tables: the same on every rank (seed 0)
    gen = torch.Generator(device=dev).manual_seed(0)
    user_w = (torch.randn(U, d, device=dev, generator=gen) * 0.01).contiguous()
    item_w = (torch.randn(I, d, device=dev, generator=gen) * 0.01).contiguous()
    t0 = time.perf_counter()
    exchange = None
    grid_trials = None
    if sharded:
        from lgcn_amd.sharded import (BlockExchange, ItemReducer, ReducePlan, RowShards, ShardedPlan, ShardGrid,
                                      UserShards, grid_candidates, propagate_forward_reduced,
                                      propagate_forward_sharded)

        in_deg = np.bincount(graph.edge_index[1], minlength=N)
        groups = {}

        def build_grid(R, F, mode):
            """This rank's share of an R x F grid: plan, layer-0 columns, exchange, step."""
            grid = ShardGrid.build(world, rank, d_full, R, F)
            c0, c1 = grid.cols
            if grid.R == 1:
                # one row group: the rank propagates its column share of the whole graph with the
                # one-GPU plan at that width (no padded layout, no halves) — bitwise the same share
                # as the sharded plan with its own slices (tests/test_gpu_sharded.py), 6 % faster
                cplan = PropagationPlan(ei, N, chunk, side_split=U)
                uw_c, iw_c = user_w[:, c0:c1].contiguous(), item_w[:, c0:c1].contiguous()
                return dict(grid=grid, shards=None, splan=None, scheds=[cplan.schedule("fwd", c1 - c0)], ex=None,
                            mode=None, step=lambda: lgcn_amd.propagate_forward(uw_c, iw_c, cplan, K))
            if (grid.R, grid.F) not in groups:  # collective: every rank creates the column groups
                groups[(grid.R, grid.F)] = grid.exchange_group(dist)
            if str(mode).startswith("reduce"):
                # users sharded, item rows all-reduced per layer (lgcn_amd.sharded.ReducePlan);
                # *-fused: a layer's two passes as one lgcn_spmm_pair launch (+ one combine);
                # reduce-a2a*: the all_reduce as all_to_all + ordered slice sums + all_gather
                ushards = UserShards.build(in_deg, U, grid.R)
                rplan = ReducePlan(ei, ushards, grid.row_group, c1 - c0, chunk)
                red = ItemReducer(grid.R, groups[(grid.R, grid.F)], method="a2a" if "a2a" in mode else "ring")
                x0u, x0i = user_w[:, c0:c1].contiguous(), item_w[:, c0:c1].contiguous()
                fused = mode.endswith("fused")
                return dict(grid=grid, shards=ushards, splan=rplan, scheds=[rplan.users, rplan.partial], ex=red,
                            mode=mode, x0=(x0u, x0i),
                            step=lambda: propagate_forward_reduced(x0u, x0i, rplan, K, red, fused=fused))
            shards = RowShards.build(in_deg, U, grid.R)
            splan = ShardedPlan(ei, shards, grid.row_group, c1 - c0, chunk)
            x0p = shards.to_padded(user_w[:, c0:c1].contiguous(), item_w[:, c0:c1].contiguous())
            ex = (BlockExchange(shards, grid.row_group, groups[(grid.R, grid.F)], grid.members, mode or "allgather")
                  if grid.R > 1 else None)
            return dict(grid=grid, shards=shards, splan=splan, scheds=[h.direction for h in splan.halves], ex=ex,
                        mode=mode, step=lambda: propagate_forward_sharded(x0p, splan, K, ex))

        def trial_ms(st, n=8):
            """This rank's ms per step of a candidate grid (untimed by the bench line)."""
            with torch.no_grad():
                for _ in range(2):
                    st["step"]()
                torch.cuda.synchronize()
                dist.barrier()
                t = time.perf_counter()
                for _ in range(n):
                    st["step"]()
                torch.cuda.synchronize()
            return (time.perf_counter() - t) / n * 1e3

        # the collectives the reduce grids price, timed once on this node before any trial (untimed
        # by the bench line): the first node run checks tools/project_scale.py's assumptions
        cands = ([tuple(int(v) for v in args.shard.split("x")) + (args.exchange_mode,)] if args.shard else
                 grid_candidates(world, d_full, p2p=os.environ.get("LGCN_GRID_NO_P2P") != "1"))
        for R, F, _ in cands:  # every rank creates every column group, in one order
            if R > 1 and (R, F) not in groups:
                groups[(R, F)] = ShardGrid.build(world, rank, d_full, R, F).exchange_group(dist)
        collectives = probe_collectives(dist, torch, dev, c2_collective_specs(world, d_full, I, groups, cands))
        for c in collectives:
            log(f"[rank {rank}] collective {c['name']}: {c['bytes'] / 1e6:.3f} MB over {c['ranks']} ranks, "
                f"{c['ms']} ms, bus {c['busbw_GBps']} GB/s")
        if args.shard:
            R, F = (int(v) for v in args.shard.split("x"))
            st = build_grid(R, F, args.exchange_mode)
        else:
            # the grid is picked by measurement: the compute per rank is known on one GPU
            # (tools/shard_rank_probe.py), the exchange cost only on the node's xGMI links.
            # A candidate that raises on any rank is skipped on every rank (the ranks agree through
            # one all_reduce of [ms, failed] per candidate), so one bad grid cannot end the run.
            st, best, grid_trials = None, None, {}
            p2p = os.environ.get("LGCN_GRID_NO_P2P") != "1"  # launch_with_fallback's second launch
            if not p2p and any(m == "p2p" for _, _, m in grid_candidates(world, d_full)):
                grid_trials["p2p candidates"] = "skipped (LGCN_GRID_NO_P2P=1)"
            for R, F, mode in grid_candidates(world, d_full, p2p=p2p):
                name = f"{R}x{F}" + (f"/{mode}" if mode else "")
                cand, ms, failed = None, 0.0, 0.0
                try:
                    cand = build_grid(R, F, mode)
                    ms = trial_ms(cand)
                except Exception as e:  # noqa: BLE001 — logged, agreed on, skipped
                    failed = 1.0
                    log(f"[rank {rank}] grid trial {name} failed: {type(e).__name__}: {e}")
                    torch.cuda.synchronize()
                agree = torch.tensor([ms, failed], dtype=torch.float64, device=dev)
                dist.all_reduce(agree, op=dist.ReduceOp.MAX)
                ms, failed = float(agree[0].item()), bool(agree[1].item())
                if failed:
                    grid_trials[name] = "failed"
                    cand = None
                    torch.cuda.empty_cache()
                    continue
                grid_trials[name] = round(ms, 4)
                log(f"[rank {rank}] grid trial {name}: {ms:.3f} ms per step")
                if best is None or ms < best:
                    st, best = cand, ms
                else:
                    del cand
                torch.cuda.empty_cache()
            if st is None:
                raise SystemExit("every grid candidate failed")
        del user_w, item_w
        grid, shards, splan, exchange, step = st["grid"], st["shards"], st["splan"], st["ex"], st["step"]
        c0, c1 = grid.cols
        d = c1 - c0
        g_r = grid.row_group
        scheds = st["scheds"]
        torch.cuda.synchronize()
        if shards is None:
            log(f"[rank {rank}] grid {grid.R}x{grid.F}: all rows, columns [{c0}, {c1}) with the one-GPU plan at "
                f"width {d}, {time.perf_counter() - t0:.2f} s")
        elif str(st["mode"]).startswith("reduce"):
            ua, ub_ = shards.users(g_r)
            log(f"[rank {rank}] grid {grid.R}x{grid.F} reduce: row group {g_r} (users {ub_ - ua} of {U}, all {I} "
                f"items from {splan.n_sub} edges), columns [{c0}, {c1}), {time.perf_counter() - t0:.2f} s")
        else:
            ua, ub_ = shards.user_rows(g_r)
            ia, ib_ = shards.item_rows(g_r)
            log(f"[rank {rank}] grid {grid.R}x{grid.F}{' ' + st['mode'] if st['mode'] else ''}: row group {g_r} "
                f"(users {ub_ - ua} of {U}, items {ib_ - ia} of {I}), columns [{c0}, {c1}); padded N {shards.NP}; "
                f"{'sliced' if splan.sliced else 'plain'} halves, {time.perf_counter() - t0:.2f} s")
    else:
        # side_split = U: rows gathering the item table run first, then rows gathering the user table
        plan = PropagationPlan(ei, N, chunk, side_split=U)
        # the schedule the forward runs at this width: source-sliced (one item-pass launch per slice
        # per layer) when lgcn_amd.plan.slice_bytes_for enables it, else the plain item list
        sched = plan.schedule("fwd", d)
        scheds = [sched]
        torch.cuda.synchronize()
        n_sl = sched.n_launches if isinstance(sched, SlicedDirection) else 1
        log(f"[rank {rank}] plan: {plan.fwd.n_items} items, {plan.fwd.n_splits} split rows, "
            f"{plan.fwd.n_partials} partials, {plan.nbytes() / 1e6:.0f} MB; "
            f"{n_sl} source slice(s) per layer, {sched.n_splits} chunked rows ({time.perf_counter() - t0:.2f} s)")

        def step():
            return lgcn_amd.propagate_forward(user_w, item_w, plan, K)

    with torch.no_grad():
        for _ in range(args.warmup):
            step()
        settle = settle_warmup(step, torch, dist if distributed else None, dev)
        sliced = isinstance(scheds[0], SlicedDirection)
        # (the ride layout is built by the first forward, so this is known after the warm-up)
        riding = (sliced and K > 1 and lgcn_amd.tuning.get().slice_ride
                  and bool(getattr(scheds[0], "_ride", None)))
        # the brackets sample every TIMER_EVERY-th timed step: the riding one-GPU forward brackets a
        # whole step's item-pass launches (2 events; ~0.4 % of a step when every step carries them),
        # the other schedules each layer's launches (~1.5 % when every step carries them)
        every = TIMER_EVERY
        timer = LaunchTimer()
        lgcn_amd.set_launch_timer(timer)
        if exchange is not None:
            exchange.bytes = 0
        step_ev = [] if args.step_times else None
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            timer.active = i % every == 0
            if step_ev is not None:
                step_ev.append(torch.cuda.Event(enable_timing=True))
                step_ev[-1].record(torch.cuda.current_stream())
            step()
        host_s = time.perf_counter() - t0  # the host's own time to issue the steps (diagnostic)
        if step_ev is not None:
            step_ev.append(torch.cuda.Event(enable_timing=True))
            step_ev[-1].record(torch.cuda.current_stream())
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        timer.active = False
        lgcn_amd.set_launch_timer(None)

    kernel_ms = timer.mean_ms()  # one item-pass launch, averaged over the timed region
    kernel_ms_basis = None
    if kernel_ms is None:  # a path without launch brackets: the step's mean per item-pass launch
        n_launch = sum(schedule_traffic(sc, N, d)[1] for sc in scheds) * K
        kernel_ms = elapsed / args.steps * 1e3 / max(1, n_launch)
        kernel_ms_basis = "no launch brackets on this path: ms_per_step / item-pass launches per step"
    if distributed:
        t = torch.tensor([elapsed, kernel_ms, host_s], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms, host_s = float(t[0].item()), float(t[1].item()), float(t[2].item())

    # one graph in every configuration: C2 on an R x F grid / C5 column-sharded over the ranks
    value = K * E * args.steps / elapsed
    # bytes of one middle layer's item pass (this rank's rows), spread over its launches
    comp_layer, launches, e_mine, n_mine, items_mine = 0, 0, 0, 0, 0
    for sc in scheds:
        b, n, e_s, r_s, it = schedule_traffic(sc, N, d)
        comp_layer, launches, e_mine, n_mine = comp_layer + b, launches + n, e_mine + e_s, n_mine + r_s
        items_mine += it
    comp_launch = comp_layer / launches
    # SURVEY §8d's no-reuse algorithmic bytes (every gathered row counted per edge) of this rank's rows
    alg_launch = (e_mine * (4 * d + 8) + n_mine * (4 * d + 8)) / launches
    if c5:
        workload = f"C5_synthetic_10Mx1M_5e8_K{K}_d{d_full}" + ("" if args.scale == 1.0 else f"_scale{args.scale}")
    else:
        workload = f"C2_ml25m_shaped_K{K}_d{d_full}" + ("" if args.scale == 1.0 else f"_scale{args.scale}")
        if sharded:
            workload += f"_grid{grid.R}x{grid.F}"
    kernel_name = (f"k_spmm_vec<{kernel_lpr(d)},sliced> (lgcn_spmm_run_slices, {launches} source-slice "
                   f"launches per layer)" if sliced else f"k_spmm_vec<{kernel_lpr(d)}> (lgcn_spmm_items)")
    if riding:
        kernel_name = (f"k_spmm_vec / k_spmm_ride<{kernel_lpr(d)},sliced> (lgcn_spmm_run_slices_ride, {launches} "
                       f"source-slice launches per layer, two of them carrying the split-row combine)")
    graph_stats = (graph.degree_stats() if graph is not None else {"num_nodes": N, "num_edges": E})
    signature = traffic_signature(workload, kernel_name, launches, items_mine, e_mine, graph_stats)
    traffic, stale = load_traffic(signature)
    basis = "pmc_memory_side" if traffic else "compulsory"
    achieved = (traffic if traffic else comp_launch) / (kernel_ms * 1e-3) / 1e9
    result = {
        "metric": f"edges propagated/sec (K={K}, d={d_full})",
        "value": value,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "warmup_settle": settle,
        "ms_per_step": elapsed / args.steps * 1e3,
        # the slowest rank's host time to issue the timed steps (a host-bound rank shows it near ms_per_step)
        "host_issue_ms_per_step": host_s / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": ("synthetic (seeded 10M x 1M Zipf bipartite graph generated on device; random N(0,0.01) embeddings)"
                 if c5 else "synthetic (seeded ML-25M-shaped bipartite graph, one graph for all ranks; random "
                            "N(0,0.01) embeddings)"),
        "config": {"workload": workload, "num_users": U, "num_items": I, "num_edges": E, "layers": K, "dim": d_full,
                   "chunk": chunk, "graphs": 1, "degree_stats": graph_stats,
                   "graph_generator": (f"synth.bipartite_device seed 0" if c5 else
                                       f"synth.ml25m_shaped seed 0 (user Zipf alpha {synth.ML25M_USER_ALPHA}, "
                                       f"offset {synth.ML25M_USER_OFFSET})"),
                   "parallelism": (f"feature-sharded over {world} GPU(s): {d} columns each, full plan per rank, "
                                   "no collective") if c5 else
                                  (f"{grid.R} row groups x {grid.F} column groups over {world} GPUs (reduce): each "
                                   f"rank propagates {d} of {d_full} columns of one edge-balanced user range and "
                                   f"the partial sums of every item row over the edges its users source; the item "
                                   f"partials are all-reduced within the column group once per layer "
                                   f"({args.dist_backend}, overlapped with the user pass and the next partial pass); "
                                   f"column groups exchange nothing; within 1e-5 per row of the 1-GPU result"
                                   if sharded and str(st["mode"]).startswith("reduce") else
                                   f"{grid.R} row groups x {grid.F} column groups over {world} GPUs: each rank "
                                   f"propagates {d} of {d_full} columns of one edge-balanced destination row range "
                                   f"(whole graph and whole column share of the table on every rank); " +
                                   (f"ranks of a column group exchange each exchanged layer's two row blocks "
                                    f"({args.dist_backend} {'all_gather' if st['mode'] == 'allgather' else 'sends to every peer'}"
                                    f"), each overlapped with the other half-layer; " if grid.R > 1 else "") +
                                   "column groups exchange nothing; " +
                                   ("bitwise the 1-GPU result" if grid.R == 1 else
                                    "within 1e-5 per row of the sliced 1-GPU result (bitwise the 1-GPU plain "
                                    "schedule at chunk 128)")
                                   if sharded else "single GPU")},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "basis": basis,
                     "traffic_unused_because": stale, "signature": signature,
                     "kernel": kernel_name,
                     "kernel_ms": kernel_ms,
                     "kernel_ms_sampled": kernel_ms_basis or (f"HIP events around all K layers' item-pass launches of every "
                                           f"{TIMER_EVERY}th timed step (the last combine launch outside), divided "
                                           f"by their count" if riding and not sharded else
                                           f"HIP events around each layer's launches, every {TIMER_EVERY}th timed step"),
                     "launches_x_kernel_ms_over_step": launches * K * kernel_ms / (elapsed / args.steps * 1e3),
                     "launches_per_layer": launches,
                     "compulsory_bytes_per_launch": comp_launch,
                     "traffic_over_compulsory": (traffic / comp_launch) if traffic else None,
                     "algorithmic_bytes_per_launch": alg_launch,
                     "effective_GBps": alg_launch / (kernel_ms * 1e-3) / 1e9,
                     # second efficiency figure: the C2 table is L2 / Infinity-Cache
                     # resident, so the item pass is bound by its L1->L2 request path, not HBM; the
                     # gathered source rows per second against the guide's fully L2-resident gather
                     # rate (MI355X_MICROARCH.md 'Indexed rows: gather into LDS': 66-73 GB/s per CU,
                     # 16.8-18.8 TB/s chip-wide; the upper end is the peak used)
                     "gathered_rows": {"achieved": e_mine * 4 * d / launches / (kernel_ms * 1e-3) / 1e9,
                                       "peak": GATHER_L2_PEAK_GBS, "unit": "GB/s",
                                       "frac": e_mine * 4 * d / launches / (kernel_ms * 1e-3) / 1e9
                                       / GATHER_L2_PEAK_GBS}},
        "cpu_baseline": None,
    }
    if sliced:
        result["config"]["hub_chunk_sliced"] = sliced_chunk(chunk)
    if args.tuned:
        result["config"]["tuning"] = args.tuned  # the source-sliced schedule's hub chunk
    if grid_trials is not None:
        result["config"]["grid_trials_ms_per_step"] = grid_trials
    if sharded:
        result["collectives"] = collectives
        result["projection"] = project_chosen_grid(st, K, collectives, elapsed / args.steps * 1e3, torch, dist)
    if step_ev is not None:
        series = [round(a.elapsed_time(b), 5) for a, b in zip(step_ev, step_ev[1:])]
        result["step_ms"] = series
        log(f"[rank {rank}] per-step ms: {series}")
    if exchange is not None:
        if str(st["mode"]).startswith("reduce"):
            result["exchange"] = {"mode": st["mode"], "all_reduces_per_step": K - 1, "reduce_scatters_per_step": 1,
                                  "MB_received_per_rank_per_step": exchange.bytes / args.steps / 1e6}
        else:
            result["exchange"] = {"mode": exchange.mode, "block_exchanges_per_step": 2 * (K - 1),
                                  "MB_received_per_rank_per_step": exchange.bytes / args.steps / 1e6}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if c5:
            # C5 does not fit a CPU run: the same generator at 1/100 scale (5e6 edges), K and d of C5
            del ei, user_w, item_w
            torch.cuda.empty_cache()
            from lgcn_amd.synth import BipartiteGraph

            sc = 0.01 * args.scale
            su, si = int(synth.C5_USERS * sc), int(synth.C5_ITEMS * sc)
            sample = synth.bipartite_device(su, si, int(synth.C5_PAIRS * sc), seed=0, device=dev).cpu().numpy()
            result["cpu_baseline"] = cpu_baseline(BipartiteGraph(su, si, sample), K, d_full, seconds_budget=10.0,
                                                  label=f"C5-generator-at-1/100-scale ({su} x {si})")
        else:
            result["cpu_baseline"] = cpu_baseline(graph, K, d)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


def harness_times(batches, U, I, K, d, dev, epochs=2):
    """ms per step of utils.train_test.train() both ways: the default (the fused batch step,
    lgcn_amd.harness) and tuning harness_fused=False (autograd + torch Adam + clip_grad_norm_); the last
    of `epochs` epochs is timed (the first builds the batch plans and captures the graphs)."""
    import torch

    from models.light_gcn import LightGCN
    from utils import train_test as TT

    from lgcn_amd import tuning

    class Fresh:
        """a loader that collates a new edge_index tensor every iteration (the reference's PyG
        DataLoader does), on the host (train() moves it) or on the device: the fused step finds
        each batch's state by content"""

        def __init__(self, where):
            from data.dataset_handler import Data

            self.Data = Data
            self.src = [b.edge_index.cpu() for b in batches] if where == "host" else [b.edge_index for b in batches]

        def __len__(self):
            return len(self.src)

        def __iter__(self):
            for ei in self.src:
                yield self.Data(edge_index=ei.clone(), num_nodes=batches[0].num_nodes)

    out = {}
    for name, fused, loader in (("fused_ms_per_step", True, batches),
                                ("fused_fresh_host_tensors_ms_per_step", True, Fresh("host")),
                                ("fused_fresh_device_tensors_ms_per_step", True, Fresh("device")),
                                ("reference_loop_ms_per_step", False, batches)):
        with tuning.tuned(harness_fused=fused):
            torch.manual_seed(0)
            model = LightGCN(U, I, num_layers=K, dim_h=d).to(dev)
            opt = torch.optim.Adam(model.parameters(), lr=1e-3)
            for e in range(epochs):
                torch.cuda.synchronize()
                t = time.perf_counter()
                TT.train(model, opt, loader, dev)
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t) / len(batches) * 1e3
            out[name] = ms
            out[name.replace("_ms_per_step", "_path")] = TT.LAST_TRAIN_PATH
            del model, opt
    out["note"] = ("utils.train_test.train() per step over one epoch of the bench's batches (the second of two), "
                   "torch.optim.Adam(lr=1e-3) + clip 1, loss read once per epoch; includes the epoch-end flush; "
                   "fused_fresh_*_tensors: the loader yields a new edge_index per batch every epoch, as the "
                   "reference's PyG DataLoader does (each batch's state found by a digest of its bytes: XXH3 on the "
                   "host for a host tensor; for a device tensor lgcn_digest128 on a side stream, started one "
                   "batch ahead, no sync per batch)")
    return out


def run_train(args):
    """C3 (1 GPU) / C4 (N GPUs): Cluster-GCN training of LightGCN K=3, d=128 on the ML-25M-shaped
    graph: 90/5/5 directed split, train graph cut into --parts parts by the host LDG partitioner,
    --parts-per-batch parts per step (union of intra-part edges), BPR loss, backward through the
    HIP propagation, clip_grad_norm_(1), Adam(1e-3). N ranks = data parallel: disjoint batches per
    rank; with the default row-lazy Adam the ranks all_gather only their nonzero gradient rows
    (lgcn_amd.distributed.RowExchange); --dense-adam all_reduces both dense gradient tables.
    value = K * (batch edges summed over ranks) / wall time."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from data.dataset_handler import Data
    from lgcn_amd import cluster, synth
    from lgcn_amd import distributed as D
    from models.light_gcn import LightGCN
    from utils.train_test import bpr_loss, compute_embeddings

    apply_tune(args.tuned)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if world > 1:
        init_dist(args.dist_backend, dev)
    K = args.layers if args.layers is not None else 3
    d = args.dim if args.dim is not None else 128
    t0 = time.perf_counter()
    if args.graph == "planted":  # ML-25M-sized with 1024 planted communities: big intra-part batches
        g, _ = synth.planted_ml25m(1024, scale=args.scale)
    else:
        g = synth.ml25m_shaped(seed=0, scale=args.scale)  # one graph, replicated tables (DP)
    U, I, N = g.num_users, g.num_items, g.num_nodes
    train_ei = synth.train_split(g.edge_index, 0.9, seed=0)
    n_tr = train_ei.shape[1]
    q = args.parts_per_batch
    _, f_intra, lists = cluster.cluster_batches(train_ei, N, args.parts, q)
    batches = [Data(edge_index=torch.from_numpy(ei).to(dev), num_nodes=N) for ei in lists]
    log(f"[rank {rank}] train graph E={n_tr} parts={args.parts} f_intra={f_intra:.4f} "
        f"batches={len(batches)} mean E_batch={np.mean([b.edge_index.shape[1] for b in batches]):.0f} "
        f"({time.perf_counter() - t0:.1f} s)")
    torch.manual_seed(0)
    model = LightGCN(U, I, num_layers=K, dim_h=d).to(dev)
    lazy = not (args.autograd or args.torch_adam or args.dense_adam)
    dp_mode = args.dp_mode if world > 1 else "replicated"
    if dp_mode == "auto":
        # tools/project_c4.py (profiles/r05zp_hybrid/): at W = 2 no mode beats one GPU by much and
        # columns keeps the one-GPU semantics; from W = 4, on batches that draw fewer negatives than
        # there are items (C3: 10k triplets, 59k items) the owner-sharded exchange is the fastest
        # (W = 8: 1.8x at 100 GB/s, 2.6x at 200), on batches whose negatives cover the items (the
        # planted graph: 180k triplets) the hybrid one (2.8x / 3.9x, owner 2.3x / 3.2x)
        mean_b = float(np.mean([int((b.edge_index[0] < U).sum()) for b in batches]))
        dp_mode = "columns" if world <= 2 else ("hybrid" if mean_b >= I else "owner")
    if dp_mode != "replicated" and not lazy:
        raise SystemExit("--dp-mode owner / columns / hybrid need the row-lazy Adam (no --autograd/--torch-adam/--dense-adam)")
    cols = None
    if dp_mode == "columns":
        from lgcn_amd.train_step import ColumnGroup

        cols = ColumnGroup(world, rank, d)
        c0, c1 = cols.cols
        full = model
        model = LightGCN(U, I, num_layers=K, dim_h=c1 - c0).to(dev)
        with torch.no_grad():
            model.user_embedding.weight.copy_(full.user_embedding.weight[:, c0:c1])
            model.item_embedding.weight.copy_(full.item_embedding.weight[:, c0:c1])
        del full
    # data parallel (W parts per Adam step): lr * sqrt(W), the rule that keeps Recall@20 and @100 on
    # the reference's (lgcn_amd.distributed.dp_lr); columns and one GPU: the reference's 1e-3
    lr = D.dp_lr(1e-3, world) if (world > 1 and cols is None and args.dp_lr == "sqrt") else 1e-3
    if args.torch_adam:
        opt = torch.optim.Adam(model.parameters(), lr=lr)
    elif lazy:
        from lgcn_amd.optim import RowLazyAdam

        opt = RowLazyAdam(model.user_embedding.weight.data, model.item_embedding.weight.data, lr=lr,
                          max_grad_norm=1)
    else:
        from lgcn_amd.optim import FusedAdam

        opt = FusedAdam(model.parameters(), lr=lr, max_grad_norm=1, capturable=not args.autograd,
                        keep_clipped_grad=False)
    params = list(model.parameters())
    torch.manual_seed(1000 + rank)

    fused = None
    exchange = None
    if dp_mode == "owner":
        from lgcn_amd import _ffi
        from lgcn_amd.owner import OwnerExchange, owner_capacity

        exchange = OwnerExchange(owner_capacity(batches, U, world, num_items=I), N, d, dev, world, rank,
                                 _ffi.load().lgcn_row_grad_norm_workspace_floats())
        log(f"[rank {rank}] owner exchange: {exchange.cap} slots per destination, blocks of "
            f"{exchange.blk * 4 / 1e6:.2f} MB, two all_to_alls per step")
    elif dp_mode == "hybrid":
        # items all_reduced densely, users' rows as record blocks (large batches)
        exchange = D.HybridExchange(D.user_exchange_capacity(batches, U), U, opt.gi, dev, world)
        log(f"[rank {rank}] hybrid exchange: {exchange.cap} user slots per rank ({exchange.blk * 4 / 1e6:.2f} MB "
            f"record block) + the item gradient table ({I * d * 4 / 1e6:.1f} MB) all_reduced per step")
    elif dp_mode == "replicated" and lazy and (world > 1 or args.exchange):
        # row-sparse DP gradient exchange: all_gather of each rank's nonzero gradient rows
        cap = D.exchange_capacity(batches, U)
        exchange = D.RowExchange(cap, N, d, dev, world)
        log(f"[rank {rank}] row exchange: {exchange.cap} slots per rank, one all_gather of "
            f"{exchange.blk * 4 / 1e6:.1f} MB per rank per step "
            f"(dense all_reduce: {N * d * 4 / 1e6:.1f} MB)")
    if not args.autograd:
        from lgcn_amd.train_step import FusedTrainStep

        fused = FusedTrainStep(model, opt, world=world if cols is None else 1,
                               graphs=not args.no_graphs and not args.torch_adam,
                               lazy=lazy, exchange=exchange, cols=cols,
                               neg_seed=(7 if cols is not None else 1000 + rank) if dp_mode != "replicated" else None)

    collectives = None
    if world > 1:  # what this mode exchanges, timed on the node before the warm-up (untimed)
        max_b = max(int((b.edge_index[0] < U).sum()) for b in batches)
        collectives = probe_collectives(dist, torch, dev, c4_collective_specs(world, dp_mode, exchange, cols, I, d,
                                                                              max_b))

    def step(bidx, nxt=None):
        batch = batches[bidx]
        if fused is not None:
            if dp_mode == "owner":
                fused.step(batch, batches[nxt] if nxt is not None else None)
            else:
                fused.step(batch)
            return batch.edge_index.shape[1]
        opt.zero_grad()
        loss = bpr_loss(*compute_embeddings(model, batch, dev))
        loss.backward()
        D.allreduce_grads(params, world)
        if args.torch_adam:
            torch.nn.utils.clip_grad_norm_(params, max_norm=1)
        opt.step()
        return batch.edge_index.shape[1]

    # column-sharded ranks all step the one schedule (the one-GPU order); the DP modes split it
    share = (D.rank_share(len(batches), 1, 0, seed=0, epoch=0) if cols is not None else
             D.rank_share(len(batches), world, rank, seed=0, epoch=0))

    def nxt_of(i, last):
        """the batch index of step i + 1 (owner mode fetches its rows), None after an epoch's end
        (sync() makes every row current there) or the run's last step"""
        return None if (i + 1) % len(share) == 0 or i + 1 == last else share[(i + 1) % len(share)]

    n_warm = max(args.warmup, 2 * len(share))
    for i in range(n_warm):  # warm-up builds every batch's plan
        step(share[i % len(share)], nxt_of(i, n_warm))
        if fused is not None and ((i + 1) % len(share) == 0 or i + 1 == n_warm):
            fused.sync()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    edges = 0
    if exchange is not None:
        exchange.bytes = 0
    for i in range(args.steps):
        edges += step(share[i % len(share)], nxt_of(i, args.steps))
        # row-lazy Adam: parameters are made current once per epoch (as evaluation needs them),
        # inside the timed region
        if fused is not None and ((i + 1) % len(share) == 0 or i + 1 == args.steps):
            fused.sync()
    host_s = time.perf_counter() - t0  # the host's own time to issue the steps (no sync inside)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if fused is not None:
        fused.check_overflow()  # outside the timed region: one host read per batch state
    if world > 1:
        t = torch.tensor([elapsed, edges], dtype=torch.float64, device=dev)
        tt = t.clone()
        dist.all_reduce(t[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(tt[1:], op=dist.ReduceOp.SUM)
        # column-sharded: every rank propagated the same batches (d / W columns each): count them once
        elapsed, edges = float(t[0].item()), float(tt[1].item()) / (world if cols is not None else 1)
    result = {
        "metric": f"training edges propagated/sec (Cluster-GCN, K={K}, d={d})",
        "value": K * edges / elapsed, "unit": "edges/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "host_issue_ms_per_step": host_s / args.steps * 1e3,
        "scaling": "strong" if cols is not None else "weak", "vs_baseline": None, "dtype": "fp32",
        "data": ("synthetic (seeded ML-25M-sized graph with 1024 planted communities, 90/5/5 directed split)"
                 if args.graph == "planted" else "synthetic (seeded ML-25M-shaped graph, 90/5/5 directed split)"),
        "config": {"workload": f"C{3 if world == 1 else 4}_cluster_gcn_train" + ("_planted" if args.graph == "planted" else ""),
                   "parts": args.parts, "mean_batch_edges": float(np.mean([b.edge_index.shape[1] for b in batches])),
                   "optimizer": ("torch Adam + clip_grad_norm_" if args.torch_adam else
                                 "lgcn RowLazyAdam (exact row-lazy Adam + clip, flushed each epoch)" if lazy else
                                 "lgcn FusedAdam (clip fused)"),
                   "step": "autograd (reference ops)" if args.autograd else
                           ("fused sparse step" + ("" if (args.no_graphs or args.torch_adam) else ", hipGraph per batch")),
                   "parts_per_batch": q, "f_intra": f_intra, "layers": K, "dim": d, "num_users": U,
                   "num_items": I, "train_edges": n_tr,
                   "batch_plan_chunks": sorted({_batch_chunk_for(int(b.edge_index.shape[1])) for b in batches}),
                   "parallelism": (f"columns{world}: every rank the same batches and negatives on {d // world} of "
                                   f"{d} columns; one all_reduce of the triplets' [B, 6] dots/norms and one "
                                   f"all_gather of the clip norm's partials per step (the one-GPU step's semantics)"
                                   if cols is not None else
                                   f"dp{world}: disjoint part batches per rank, " +
                                   ("owner-sharded row-lazy Adam (row r owned by rank r % W): gradient rows to their "
                                    "owners and the next step's rows back, two all_to_alls + the clip norm's "
                                    "partials per step" if dp_mode == "owner" else
                                    "item gradient table all_reduced densely, users' rows all-gathered as records, "
                                    "every item row and the users' union stepped" if dp_mode == "hybrid" else
                                    "row-sparse gradient exchange (one all_gather per step of each rank's nonzero rows and their ids), "
                                    "row-lazy Adam on the union" if exchange is not None else
                                    "RCCL all_reduce of embedding grads" if world > 1 else "single GPU"))},
    }
    if args.tuned:
        result["config"]["tuning"] = args.tuned
    if exchange is not None and hasattr(exchange, "bytes"):
        result["exchange"] = {"mode": dp_mode, "MB_received_per_rank_per_step": exchange.bytes / args.steps / 1e6}
    if collectives is not None:
        result["collectives"] = collectives
    if world == 1 and not args.no_harness:
        # what a user of the reference harness gets: utils.train_test.train() over one epoch of the
        # same batches with the reference's torch Adam(1e-3) (clip 1 inside), routed to the fused
        # step (lgcn_amd.harness), next to the reference-style loop it replaces (untimed by the line)
        result["harness"] = harness_times(batches, U, I, K, d, dev)
    # what the chosen mode's training semantics are held to (tests/test_gpu_dp_recall.py, C1 size)
    result["recall_parity"] = (
        {"mode": "columns", "status": "exact schedule: the one-GPU step's batches, negatives and Adam steps on d/N "
                                      "columns each; Recall@20/@100 equal the one-GPU run's (asserted within "
                                      "+-0.002 of the reference harness)"}
        if cols is not None else
        {"mode": dp_mode, "lr": lr,
         "status": f"data parallel: W = {world} parts per Adam step at lr 1e-3 * sqrt(W) (--dp-lr sqrt); C1 size "
                   "at W = 8: |dRecall@20| 0.00015, |dRecall@100| 0.00025 (both asserted within +-0.002); at "
                   "lr 1e-3 (--dp-lr same) 0.0015 / 0.0030 (Recall@100 outside)"}
        if world > 1 else
        {"mode": "single GPU", "status": "the reference schedule; C1 size: the GPU-trained tables give the CPU "
                                        "oracle's Recall@20/@100 exactly; GPU evaluate() with recall_ties='cpu' "
                                        "equals the CPU reference, with the default GPU tie rule it equals the "
                                        "oracle tables under that rule (tests/test_gpu_training.py)"})
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
