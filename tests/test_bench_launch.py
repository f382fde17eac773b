"""bench.py as its own launcher: `python bench.py --gpus N` outside torchrun starts N rank
processes (the driver's SCALE run calls it that way). CPU only: a stand-in rank program checks the
environment each rank gets, the relay of rank 0's JSON line and the failure path; the rendezvous
itself is exercised with a world-2 gloo barrier."""
import importlib.util
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


RANK_PROGRAM = r"""
import json, os, sys
import torch.distributed as dist
keys = ["RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"]
env = {k: os.environ.get(k) for k in keys}
dist.init_process_group("gloo")
dist.barrier()
fail = os.environ.get("FAIL_RANK")
if fail is not None and int(os.environ["RANK"]) == int(fail):
    sys.exit(3)
if int(os.environ["RANK"]) == 0:
    print(json.dumps({"env": env, "world": dist.get_world_size(), "argv": sys.argv[1:]}), flush=True)
dist.destroy_process_group()
"""


def test_child_envs_match_torchrun():
    b = _bench()
    envs = b.child_envs(4, 29555, base={"PATH": "/usr/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    for e in envs:
        assert e["WORLD_SIZE"] == "4" and e["LOCAL_WORLD_SIZE"] == "4"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29555"
        assert e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and e["PATH"] == "/usr/bin"


def test_launch_relays_rank0_json(tmp_path, capfd):
    b = _bench()
    prog = tmp_path / "rank.py"
    prog.write_text(RANK_PROGRAM)
    os.environ.pop("FAIL_RANK", None)
    rc = b.launch_ranks(2, ["--gpus", "2", "--steps", "3"], script=prog)
    assert rc == 0
    out = capfd.readouterr().out.strip().splitlines()
    assert len(out) == 1
    rec = json.loads(out[0])
    assert rec["world"] == 2 and rec["env"]["RANK"] == "0" and rec["env"]["WORLD_SIZE"] == "2"
    assert rec["argv"] == ["--gpus", "2", "--steps", "3"]


def test_launch_fails_when_a_rank_fails(tmp_path, monkeypatch):
    b = _bench()
    prog = tmp_path / "rank.py"
    prog.write_text(RANK_PROGRAM)
    monkeypatch.setenv("FAIL_RANK", "1")
    assert b.launch_ranks(2, [], script=prog) == 3


def test_bench_main_becomes_the_launcher(tmp_path):
    """`python bench.py --gpus 2` with no WORLD_SIZE re-runs itself as 2 ranks; a bad flag in the
    ranks' argv makes every rank fail, and the launcher returns non-zero without touching a GPU."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--config", "c2", "--shard", "bad"],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode != 0
    assert "launch: 2 rank processes" in r.stderr


def test_traffic_entry_needs_a_matching_signature(tmp_path, monkeypatch):
    """roofline.traffic comes from profiles/pmc_traffic.json only when the entry's recorded plan
    signature equals the run's; any difference (kernel source, launches, graph) falls back."""
    b = _bench()
    sig = b.traffic_signature("W", "k<16>", 7, 100, 1000, {"user_max": 5})
    assert sig["kernel_source_sha16"] == b.kernel_source_sha16() and len(sig["kernel_source_sha16"]) == 16
    prof = tmp_path / "profiles"
    prof.mkdir()
    monkeypatch.setattr(b, "ROOT", tmp_path)
    assert b.load_traffic(sig)[0] is None  # no file
    (prof / "pmc_traffic.json").write_text(json.dumps({"W": {"hbm_bytes_per_launch": 123.0, "signature": sig}}))
    assert b.load_traffic(sig) == (123.0, None)
    other = dict(sig, launches_per_layer=8)
    val, why = b.load_traffic(other)
    assert val is None and "launches_per_layer" in why
    (prof / "pmc_traffic.json").write_text(json.dumps({"W": {"hbm_bytes_per_launch": 123.0}}))  # no signature
    assert b.load_traffic(sig)[0] is None


def test_committed_c2_entry_matches_its_kernel_source():
    """The committed C2 PMC entry was measured on the kernel source in the tree."""
    b = _bench()
    ent = json.loads((ROOT / "profiles" / "pmc_traffic.json").read_text())["C2_ml25m_shaped_K3_d64"]
    assert ent["signature"]["kernel_source_sha16"] == b.kernel_source_sha16()


def test_launcher_stops_its_ranks_when_stopped(tmp_path):
    """SIGTERM to the launcher (a driver timeout) stops every rank; none is left running."""
    import signal
    import time

    prog = tmp_path / "sleeper.py"
    pids = tmp_path / "pids"
    pids.mkdir()
    prog.write_text("import os, time, pathlib\n"
                    f"pathlib.Path({str(pids)!r}, str(os.getpid())).write_text('x')\n"
                    "time.sleep(600)\n")
    launcher = tmp_path / "launch.py"
    launcher.write_text("import importlib.util, sys\n"
                        f"spec = importlib.util.spec_from_file_location('b', {str(ROOT / 'bench.py')!r})\n"
                        "b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)\n"
                        f"sys.exit(b.launch_ranks(3, [], script={str(prog)!r}))\n")
    p = subprocess.Popen([sys.executable, str(launcher)])
    deadline = time.time() + 60
    while len(list(pids.iterdir())) < 3 and time.time() < deadline:
        time.sleep(0.2)
    assert len(list(pids.iterdir())) == 3
    p.send_signal(signal.SIGTERM)
    assert p.wait(timeout=60) == 128 + signal.SIGTERM
    time.sleep(0.5)
    for f in pids.iterdir():
        with pytest.raises(ProcessLookupError):
            os.kill(int(f.name), 0)


def _args(**kw):
    import argparse

    base = dict(gpus=8, workload="propagate", config="c2", shard=None)
    base.update(kw)
    return argparse.Namespace(**base)


@pytest.mark.parametrize("first_rc,first_out,kw,relaunched", [
    (1, [], {}, True),                          # no result: once more without the peer-send grids
    (1, [b"{}\n"], {}, False),                  # a result was relayed: never a second line
    (0, [b"{}\n"], {}, False),
    (1, [], {"gpus": 2}, False),                # no p2p candidate below 3 ranks per row group
    (1, [], {"workload": "train"}, False),
    (1, [], {"config": "c5"}, False),
    (1, [], {"shard": "4x2"}, False),
])
def test_launch_fallback_without_p2p(monkeypatch, first_rc, first_out, kw, relaunched):
    b = _bench()
    monkeypatch.delenv("LGCN_GRID_NO_P2P", raising=False)
    calls = []

    def fake_launch(n, argv, relayed):
        calls.append(os.environ.get("LGCN_GRID_NO_P2P"))
        if len(calls) == 1:
            relayed.extend(first_out)
            return first_rc
        relayed.append(b"{}\n")
        return 0

    rc = b.launch_with_fallback(_args(**kw), launch=fake_launch)
    assert calls == ([None, "1"] if relaunched else [None])
    assert rc == (0 if relaunched else first_rc)


def _collectives_worker(rank, world, port, out):
    import sys

    import torch
    import torch.distributed as dist

    sys.path[:0] = [str(ROOT), str(ROOT / "movie-recommender-system-with-gnns_amd")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b = _bench()
    cpu = torch.device("cpu")
    # the C2 4x2-shaped specs at world 2: one 1 x 2 "grid" has no exchange, so price a 2 x 1 group
    specs = b.c2_collective_specs(world, 64, 3000, {(2, 1): None}, [(2, 1, "reduce"), (1, 2, None)])
    specs += b.c4_collective_specs(world, "hybrid", type("X", (), {"blk": 1000})(), None, 3000, 8, 500)
    rec = b.probe_collectives(dist, torch, cpu, specs, reps=3, sync=lambda: None)
    if rank == 0:
        with open(out, "w") as f:
            json.dump(rec, f)
    dist.destroy_process_group()


def test_collectives_probe_schema(tmp_path):
    """bench.py --gpus N times the collectives its projections price (untimed,
    before the grid trials / the training warm-up) and writes them into the JSON line: name, op,
    ranks, bytes, ms (max over ranks), bus and algorithm bandwidth; a collective the backend lacks
    is recorded as failed on every rank instead of ending the run. World-2 gloo rehearsal."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "coll.json")
    mp.spawn(_collectives_worker, args=(2, port, out), nprocs=2, join=True)
    with open(out) as f:
        rec = json.load(f)
    names = [r["name"] for r in rec]
    assert names == ["2x1_items_all_reduce", "2x1_items_reduce_scatter", "2x1_items_all_to_all", "2x1_items_all_gather",
                     "2x1_latency_all_reduce_8B", "world_latency_all_reduce_8B", "hybrid_items_all_reduce",
                     "hybrid_users_all_gather", "world_latency_all_reduce_8B"]
    for r in rec:
        assert set(r) >= {"name", "op", "ranks", "bytes", "ms", "busbw_GBps", "algbw_GBps"}, r
        assert r["ranks"] == 2 and r["bytes"] >= 8
        if r.get("failed"):
            assert r["ms"] is None and r["busbw_GBps"] is None
        else:
            assert r["ms"] > 0 and r["busbw_GBps"] > 0
    by = {r["name"]: r for r in rec}
    assert not by["2x1_items_all_reduce"].get("failed")  # gloo has all_reduce
    assert by["2x1_items_all_reduce"]["bytes"] == 3000 * 64 * 4
    # all_reduce's bus bytes: 2 (n-1)/n of the buffer
    r = by["2x1_items_all_reduce"]
    assert abs(r["busbw_GBps"] - r["algbw_GBps"]) <= 0.02 * r["algbw_GBps"] + 0.01
