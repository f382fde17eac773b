"""Launch programs (include/lgcn.h ABI 11, lgcn_amd.train_step.StepProgram): a captured hipGraph
issued as plain launches on the stream. The one-GPU fused Cluster-GCN step (reference
utils/train_test.py:86-101) is captured once per batch and, by default, run this way instead of
hipGraphLaunch. These tests hold the program to the graph replay and to the eager
step bitwise: every loss, both tables and both Adam moments."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


class _Batch:
    def __init__(self, ei):
        self.edge_index = ei


def _hip():
    lib = ctypes.CDLL("libamdhip64.so")
    lib.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    lib.hipMemsetAsync.restype = ctypes.c_int
    return lib


def _bufs(gpu, n):
    torch.manual_seed(3)
    return (torch.randn(n, device=gpu), torch.randn(n, device=gpu), torch.zeros(n, device=gpu),
            torch.full((n,), 7, dtype=torch.int32, device=gpu))


def _seq(gpu, n, copy):
    from lgcn_amd import _ffi

    lib = _ffi.load()
    hip = _hip()

    def run(a, b, c, z):
        s = torch.cuda.current_stream(gpu).cuda_stream
        a.mul_(1.5).add_(b)                                                            # torch kernels
        _ffi.check(lib.lgcn_scale(a.data_ptr(), b.data_ptr(), n, 3.0, 0.5, s), "lgcn_scale")  # library kernel
        assert hip.hipMemsetAsync(ctypes.c_void_p(z.data_ptr()), 0, 4 * (n - 3), ctypes.c_void_p(s)) == 0  # memset
        if copy:
            c.copy_(b)                                                                 # device-to-device copy
        else:
            c.add_(b)
        z[n - 3:].add_(1)

    return run


def _program_vs_eager(gpu, copy):
    from lgcn_amd.train_step import StepProgram

    n = 4099  # not a multiple of 8: the memset has a ragged tail
    seq = _seq(gpu, n, copy)
    ref = _bufs(gpu, n)
    for _ in range(3):
        seq(*ref)
    torch.cuda.synchronize()
    got = _bufs(gpu, n)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g):
        seq(*got)
    prog = StepProgram(g)
    for _ in range(3):
        prog.replay()
    torch.cuda.synchronize()
    for x, y in zip(ref, got):
        assert torch.equal(x, y)
    return prog


def test_program_issues_kernels_and_memsets_in_order(gpu):
    """torch kernels, a library kernel and a HIP memset node, captured from one stream, run three
    times as a program: the same values as the sequence run eagerly three times (each run reads
    what the previous one wrote, so order and repetition both show)."""
    prog = _program_vs_eager(gpu, copy=False)
    assert prog.refused is None, prog.refused
    assert prog.launches >= 5


def test_program_refuses_a_copy_node_and_replays_the_graph(gpu):
    """A captured device copy has no stream-launch form here: the library refuses the graph and
    StepProgram replays it as a hipGraph — the same values."""
    prog = _program_vs_eager(gpu, copy=True)
    assert prog.refused is not None and "node type" in prog.refused
    assert prog.launches is None


def _train(gpu, mode, min_b, clip, steps=24):
    """mode: 'eager' (no capture), 'graph' (hipGraph replay), 'program' (the default)."""
    import graphs
    from lgcn_amd import cluster as C
    from lgcn_amd import tuning
    from lgcn_amd.optim import RowLazyAdam
    from lgcn_amd.train_step import FusedTrainStep, StepProgram
    from models.light_gcn import LightGCN

    U, I, ei = graphs.subsampled(U=2000, I=1000, pairs=8000, seed=4)
    part = C.partition_nodes(ei, U + I, 8)
    batches = [_Batch(torch.from_numpy(x).to(gpu)) for x in C.intra_part_edges(ei, part, 8)]
    with tuning.tuned(step_program=(mode == "program"), sorted_scatter_min_b=min_b):
        torch.manual_seed(0)
        m = LightGCN(U, I, num_layers=3, dim_h=64).to(gpu)
        opt = RowLazyAdam(m.user_embedding.weight.data, m.item_embedding.weight.data, lr=1e-2, max_grad_norm=clip)
        step = FusedTrainStep(m, opt, graphs=(mode != "eager"), lazy=True)
        losses = []
        for i in range(steps):
            torch.cuda.manual_seed(100 + i)
            losses.append(step.step(batches[i % 8]).item())
            if (i + 1) % 8 == 0:
                step.sync()
        step.sync()
        kinds = {type(getattr(st, "graph", None)).__name__ for st in step._states.values()}
        if mode == "program":
            assert kinds == {"StepProgram"}, kinds
            for st in step._states.values():
                assert isinstance(st.graph, StepProgram) and st.graph.refused is None, st.graph.refused
                assert st.graph.launches >= 8
        ea, eb = opt.exp_avg()
        sa, sb = opt.exp_avg_sq()
        return losses, [t.detach().clone() for t in (m.user_embedding.weight, m.item_embedding.weight, ea, eb, sa, sb)]


@pytest.mark.parametrize("min_b,clip", [(49152, 1.0), (1, 1.0), (49152, float("inf"))])
def test_step_program_bitwise_graph_replay_and_eager(gpu, min_b, clip):
    """The same 24 steps (3 epochs of 8 batches, flushed each epoch) eagerly, as hipGraph replays
    and as launch programs: bitwise equal losses, tables and moments. min_b = 1 puts every batch on
    the sorted negatives path (the counting-sort grouping's kernels in the program)."""
    runs = {mode: _train(gpu, mode, min_b, clip) for mode in ("eager", "graph", "program")}
    for mode in ("graph", "program"):
        assert runs[mode][0] == runs["eager"][0], mode
        for x, y in zip(runs[mode][1], runs["eager"][1]):
            assert torch.equal(x, y), mode


def _train_exchange(gpu, program: bool, steps=12):
    import graphs
    from lgcn_amd import cluster as C
    from lgcn_amd import distributed as D
    from lgcn_amd import tuning
    from lgcn_amd.optim import RowLazyAdam
    from lgcn_amd.train_step import FusedTrainStep, StepProgram
    from models.light_gcn import LightGCN

    U, I, ei = graphs.subsampled(U=2000, I=1000, pairs=8000, seed=4)
    part = C.partition_nodes(ei, U + I, 8)
    batches = [_Batch(torch.from_numpy(x).to(gpu)) for x in C.intra_part_edges(ei, part, 8)]
    cap = D.exchange_capacity(batches, U)
    with tuning.tuned(step_program=program):
        torch.manual_seed(0)
        m = LightGCN(U, I, num_layers=3, dim_h=64).to(gpu)
        opt = RowLazyAdam(m.user_embedding.weight.data, m.item_embedding.weight.data, lr=1e-2, max_grad_norm=1.0)
        step = FusedTrainStep(m, opt, graphs=True, lazy=True, exchange=D.RowExchange(cap, U + I, 64, gpu, 1))
        losses = []
        for i in range(steps):
            torch.cuda.manual_seed(100 + i)
            losses.append(step.step(batches[i % 8]).item())
        step.sync()
        if program:
            for st in step._states.values():
                for half in (st.graph, st.graph_post):
                    assert isinstance(half, StepProgram)
                    print("exchange step half:", half.launches, "launches" if half.refused is None else
                          f"replayed as a graph ({half.refused})")
        return losses, m.user_embedding.weight.detach().clone(), m.item_embedding.weight.detach().clone()


def test_exchange_step_halves_as_programs_bitwise_graph_replay(gpu):
    """The data-parallel step's two captured halves (before / after the row exchange's all_gather,
    one rank) issued as launch programs: bitwise their hipGraph replays."""
    a = _train_exchange(gpu, program=False)
    b = _train_exchange(gpu, program=True)
    assert a[0] == b[0]
    assert torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])


def test_program_orders_a_forked_capture(gpu):
    """A capture that forks onto a second stream and joins again has two parallel branches; the
    program issues them one after the other in a dependency order: the joined result equals the
    eager sequence's, three runs in a row."""
    from lgcn_amd.train_step import StepProgram

    n = 1 << 16

    def bufs():
        torch.manual_seed(5)
        return [torch.randn(n, device=gpu) for _ in range(3)]

    side = torch.cuda.Stream(gpu)

    def seq(a, b, c):
        main = torch.cuda.current_stream(gpu)
        side.wait_stream(main)
        a.mul_(0.5).add_(1.0)          # branch 1 (main stream)
        with torch.cuda.stream(side):
            b.mul_(2.0).sub_(c)        # branch 2 (side stream)
            c.add_(0.25)
        main.wait_stream(side)
        a.add_(b).mul_(c)              # the join reads both branches

    ref = bufs()
    for _ in range(3):
        seq(*ref)
    torch.cuda.synchronize()
    got = bufs()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g):
        seq(*got)
    prog = StepProgram(g)
    assert prog.refused is None, prog.refused
    assert prog.launches == 7
    for _ in range(3):
        prog.replay()
    torch.cuda.synchronize()
    for x, y in zip(ref, got):
        assert torch.equal(x, y)
