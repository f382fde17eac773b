"""Round-4 entry points and fixes, on the GPU:

* lgcn_spmm_pair (two independent plain passes per launch, the reduce-mode sharded forward's fused
  order) is bitwise the two passes issued alone, at every vector width, with and without split rows;
* lgcn_stack_mean_rows is bitwise the INIT / ADD / FINAL_ACC (K == 1: FINAL_E) epilogue sequence;
* lgcn_row_adam never reads last[] for list entries its first_b filter drops (the exchanges' -1
  padding), with `last` at the start of its own allocation;
* lgcn_adam_consts builds exactly the constants tools/markstein_check.c proves the row Adam's
  division shortcut for (host libm pow), and flags other beta2 schedules off the shortcut.
Reference: models/light_gcn.py:33-36 (LGConv layers + stack mean), utils/train_test.py:95-96 (Adam).
"""
import ctypes
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _direction(dev, ei, N, chunk, side_split):
    from lgcn_amd import _ffi
    from lgcn_amd.plan import _build_direction

    key = torch.from_numpy(ei[1]).to(dev)
    other = torch.from_numpy(ei[0]).to(dev)
    d, _, bad = _build_direction(key, other, N, chunk, side_split, None, _ffi.stream_of(dev))
    assert bad == 0
    return d


def _pass(direction, x, y, acc, part, mode, e=None, div=1.0, mul=1.0, packed=False):
    from lgcn_amd import _ffi

    N = x.shape[0]
    return _ffi.Pass(direction.items.data_ptr(), direction.n_items, direction.splits.data_ptr(), direction.n_splits,
                     direction.col.data_ptr(), direction.val.data_ptr(), x.data_ptr(), None, N,
                     _ffi.ptr(e), None, N, _ffi.ptr(y), acc.data_ptr(), None, N, _ffi.ptr(part), mode, div, mul,
                     n_split_big=direction.n_split_big if packed else -1)


@pytest.mark.parametrize("d", [4, 8, 16, 32, 64, 128, 256, 512])
@pytest.mark.parametrize("chunk,xcd,packed", [(8, "0", False), (4096, "0", False), (8, "4", False),
                                              (4096, "4", False), (8, "4", True), (2, "4", True), (8, "3", True),
                                              (8, "7", False)])
def test_spmm_pair_bitwise_single_passes(gpu, tune, d, chunk, xcd, packed):
    """xcd = tuning pair_xcds_a: the XCD-split block mapping (pass a on xcd of the 8 XCDs, b on the rest,
    while both have blocks left; 0 = a's blocks then b's) gives the same rows; packed: split rows ordered big-first (pack_split_rows) and the
    <= 16-chunk ones combined one per lane group — the same rows too (chunk 2: hub rows of
    hundreds of chunks beside small ones)."""
    import graphs

    tune(pair_xcds_a=int(xcd))
    from lgcn_amd import _ffi
    from lgcn_amd.plan import pack_split_rows
    from lgcn_amd.propagate import spmm

    U, I, ei_a = graphs.hub(U=1500, I=40, seed=1)
    N = U + I
    _, _, ei_b = graphs.subsampled(U=U, I=I, pairs=9000, seed=3)
    da = _direction(gpu, ei_a, N, chunk, U)
    db = _direction(gpu, ei_b, N, chunk, 0)
    if packed:
        nb_a, nb_b = pack_split_rows(da), pack_split_rows(db)
        assert da.n_splits > nb_a  # some small rows to pack
        if chunk == 2:
            assert nb_a > 0  # and big ones beside them
    g = torch.Generator(device=gpu).manual_seed(d)
    xa = torch.randn(N, d, device=gpu, generator=g)
    xb = torch.randn(N, d, device=gpu, generator=g)
    e = torch.randn(N, d, device=gpu, generator=g)
    lib = _ffi.load()
    outs = []
    for paired in (False, True):
        acc_a = torch.full((N, d), 7.0, device=gpu)
        acc_b = torch.full((N, d), 7.0, device=gpu)
        y_b = torch.zeros(N, d, device=gpu)
        pa_ = torch.empty((max(1, da.n_partials), d), device=gpu)
        pb_ = torch.empty((max(1, db.n_partials), d), device=gpu)
        if paired:
            pa = _pass(da, xa, None, acc_a, pa_, _ffi.EPI_STORE, packed=packed)
            pb = _pass(db, xb, y_b, acc_b, pb_, _ffi.EPI_INIT, e=e, packed=packed)
            _ffi.check(lib.lgcn_spmm_pair(ctypes.byref(pa), ctypes.byref(pb), N, d, 1, _ffi.stream_of(gpu)), "pair")
            _ffi.check(lib.lgcn_spmm_pair(ctypes.byref(pa), ctypes.byref(pb), N, d, 2, _ffi.stream_of(gpu)), "pair")
        else:
            spmm(da, N, d, (xa, None, N), None, (acc_a, None, N), None, _ffi.EPI_STORE, 1.0, 1.0, pa_)
            spmm(db, N, d, (xb, None, N), (e, None, N), (acc_b, None, N), y_b, _ffi.EPI_INIT, 1.0, 1.0, pb_)
        outs.append((acc_a.cpu(), acc_b.cpu(), y_b.cpu()))
    if chunk <= 8:
        assert da.n_splits > 0 and db.n_splits > 0
    for one, two in zip(*outs):
        assert torch.equal(one, two)


def test_spmm_pair_argument_errors(gpu):
    from lgcn_amd import _ffi

    lib = _ffi.load()
    p = _ffi.Pass()
    assert lib.lgcn_spmm_pair(None, ctypes.byref(p), 4, 8, 1, None) == _ffi.E_ARG
    assert lib.lgcn_spmm_pair(ctypes.byref(p), ctypes.byref(p), 4, 8, 0, None) == _ffi.E_ARG
    p.n_items, p.mode = 1, 9
    assert lib.lgcn_spmm_pair(ctypes.byref(p), ctypes.byref(p), 4, 8, 1, None) == _ffi.E_ARG
    assert b"bad mode" in lib.lgcn_last_error()
    p.mode, p.n_splits, p.n_split_big = 0, 2, 3
    assert lib.lgcn_spmm_pair(ctypes.byref(p), ctypes.byref(p), 4, 8, 1, None) == _ffi.E_ARG


@pytest.mark.parametrize("K", [1, 2, 3, 4])
def test_stack_mean_rows_bitwise_epilogues(gpu, K):
    """The kept-layers mean equals the epilogue sequence the one-GPU forward applies per layer."""
    from lgcn_amd import _ffi

    rows, d = 777, 32
    g = torch.Generator(device=gpu).manual_seed(K)
    e = torch.randn(rows, d, device=gpu, generator=g)
    ys = [torch.randn(rows, d, device=gpu, generator=g) * 10 ** (-k) for k in range(K)]
    div = float(K + 1)
    mul = float(np.float32(1.0 / (K + 1)))
    # numpy fp32: one correctly rounded op at a time (torch's CUDA `tensor / scalar` multiplies by
    # the scalar's reciprocal instead, which is not the epilogue's division)
    en, yn = e.cpu().numpy(), [y.cpu().numpy() for y in ys]
    acc = en + yn[0]
    for y in yn[1:]:
        acc = acc + y
    ref = torch.from_numpy((acc / np.float32(div)) * np.float32(mul)).to(gpu)
    out = torch.empty_like(e)
    arr = (ctypes.c_void_p * K)(*[y.data_ptr() for y in ys])
    lib = _ffi.load()
    _ffi.check(lib.lgcn_stack_mean_rows(e.data_ptr(), arr, K, rows, d, out.data_ptr(), div, mul,
                                        _ffi.stream_of(gpu)), "lgcn_stack_mean_rows")
    assert torch.equal(out, ref)
    assert lib.lgcn_stack_mean_rows(e.data_ptr(), arr, 9, rows, d, out.data_ptr(), div, mul, None) == _ffi.E_ARG


@pytest.mark.parametrize("mode", [0, 1, 3])
def test_row_adam_padding_never_reads_last(gpu, mode):
    """The exchanges pass -1-padded id lists with first_b = 0 on the padding. With `last` placed at
    the very start of its own allocation, a read of last[-1] would leave the allocation: the
    padded entries must be dropped before last[] is touched, and the listed rows stepped exactly
    as the same list without padding steps them."""
    from lgcn_amd import _ffi

    lib = _ffi.load()
    U, I, d = 300, 200, 64
    N = U + I
    s = _ffi.stream_of(gpu)
    consts = torch.empty((64, 4), device=gpu)
    _ffi.check(lib.lgcn_adam_consts(consts.data_ptr(), 1, 62, 1e-3, 0.9, 0.999, s), "consts")
    results = []
    for padded in (False, True):
        g = torch.Generator(device=gpu).manual_seed(5)
        p = [torch.randn(U, d, device=gpu, generator=g), torch.randn(I, d, device=gpu, generator=g)]
        gr = [torch.randn(U, d, device=gpu, generator=g), torch.randn(I, d, device=gpu, generator=g)]
        m = [torch.zeros(U, d, device=gpu), torch.zeros(I, d, device=gpu)]
        v = [torch.zeros(U, d, device=gpu), torch.zeros(I, d, device=gpu)]
        # a fresh allocation for `last` alone (a large one, so the caching allocator gives it its own
        # block start rather than a slice of a pooled segment)
        last_buf = torch.zeros(1 << 21, dtype=torch.int32, device=gpu)
        last = last_buf[:N]
        assert last.data_ptr() == last_buf.data_ptr()
        last[:U // 2] = 1
        claim = torch.full((N,), -1, dtype=torch.int32, device=gpu)
        step = torch.full((1,), 3 if mode != 3 else 4, dtype=torch.int64, device=gpu)
        ids = torch.tensor([5, 17, U + 3, 250, U + 150], dtype=torch.int64, device=gpu)
        first = torch.ones(ids.numel(), dtype=torch.uint8, device=gpu)
        if padded:
            pad = torch.full((64,), -1, dtype=torch.int64, device=gpu)
            ids = torch.cat([pad[:7], ids[:2], pad[7:20], ids[2:], pad[20:]])
            first = (ids >= 0).to(torch.uint8)
        clip = torch.tensor([1.0, 0.5], device=gpu) if mode == 3 else None
        _ffi.check(lib.lgcn_row_adam(p[0].data_ptr(), p[1].data_ptr(), gr[0].data_ptr(), gr[1].data_ptr(),
                                     m[0].data_ptr(), m[1].data_ptr(), v[0].data_ptr(), v[1].data_ptr(), U, d, None, 0,
                                     ids.data_ptr(), ids.numel(), 0, first.data_ptr(), None, 0, last.data_ptr(),
                                     claim.data_ptr(), step.data_ptr(), consts.data_ptr(), 0.1, 0.999, 0.001, 1e-8,
                                     _ffi.ptr(clip), mode, s), "lgcn_row_adam")
        torch.cuda.synchronize()
        results.append([t.cpu() for t in (*p, *m, *v, last, step)])
    for a, b in zip(*results):
        assert torch.equal(a, b)


def test_adam_consts_are_the_checked_schedule(gpu):
    """Every distinct step constant sqrt(1 - 0.999^t) the device builds equals the host-libm value
    tools/markstein_check.c proved the Markstein division for (t up to where it reaches 1.0f), and
    the step sizes equal the host formula; consts[0].x flags the schedule, and another beta2
    (np.float32(0.999) as a double) clears it."""
    from lgcn_amd import _ffi

    lib = _ffi.load()
    T = 20000
    consts = torch.zeros((T + 2, 4), device=gpu)
    s = _ffi.stream_of(gpu)
    _ffi.check(lib.lgcn_adam_consts(consts.data_ptr(), 1, T + 1, 1e-3, 0.9, 0.999, s), "consts")
    c = consts.cpu().numpy()
    assert c[0, 0] == 1.0
    t = np.arange(1, T + 2)
    host_c = np.array([np.float32(math.sqrt(1.0 - math.pow(0.999, float(k)))) for k in t], dtype=np.float32)
    host_s = np.array([np.float32(-(float(np.float32(1e-3)) / (1.0 - math.pow(0.9, float(k))))) for k in t],
                      dtype=np.float32)
    assert host_c[-1] == np.float32(1.0)  # the whole schedule is covered
    bad = np.nonzero(c[1:, 1].view(np.uint32) != host_c.view(np.uint32))[0]
    assert bad.size == 0, f"device bc2_sqrt differs from host libm at t = {(bad[:8] + 1).tolist()}"
    assert np.array_equal(c[1:, 0].view(np.uint32), host_s.view(np.uint32))
    # the reciprocal the row Adam multiplies by: fp32 1 / c, correctly rounded (ABI 6)
    assert np.array_equal(c[1:, 2].view(np.uint32), (np.float32(1.0) / c[1:, 1]).astype(np.float32).view(np.uint32))
    _ffi.check(lib.lgcn_adam_consts(consts.data_ptr(), 1, 10, 1e-3, 0.9, float(np.float32(0.999)), s), "consts")
    assert float(consts[0, 0].item()) == 0.0


@pytest.mark.parametrize("d", [4, 8, 16, 32, 64, 128, 256, 512, 6])
@pytest.mark.parametrize("chunk,packed", [(8, False), (8, True), (2, True), (4096, True)])
def test_spmm_pass_bitwise_spmm(gpu, d, chunk, packed):
    """lgcn_spmm_pass (one plain pass from an lgcn_pass_t; packed: the <= 16-chunk split rows
    combined one per lane group, pack_split_rows' order) is bitwise lgcn_spmm on the same rows —
    for every epilogue mode the reduce-mode forward uses, at vector widths and a scalar one (d=6)."""
    import graphs

    from lgcn_amd import _ffi
    from lgcn_amd.plan import pack_split_rows
    from lgcn_amd.propagate import spmm

    U, I, ei = graphs.hub(U=1500, I=40, seed=1)
    N = U + I
    da = _direction(gpu, ei, N, chunk, U)
    if packed:
        pack_split_rows(da)
    if chunk == 2:
        assert da.n_split_big > 0 and da.n_splits > da.n_split_big
    g = torch.Generator(device=gpu).manual_seed(d + chunk)
    x = torch.randn(N, d, device=gpu, generator=g)
    e = torch.randn(N, d, device=gpu, generator=g)
    part = torch.empty((max(1, da.n_partials), d), device=gpu)
    lib = _ffi.load()
    for mode in (_ffi.EPI_STORE, _ffi.EPI_INIT, _ffi.EPI_ADD, _ffi.EPI_FINAL_ACC):
        ee = (e, None, N) if mode == _ffi.EPI_INIT else None
        outs = []
        for how in ("spmm", "pass", "pass"):  # twice: nothing carried between launches
            acc = torch.full((N, d), 0.5, device=gpu)
            y = torch.zeros(N, d, device=gpu)
            if how == "spmm":
                spmm(da, N, d, (x, None, N), ee, (acc, None, N), y, mode, 4.0, 1.0, part)
            else:
                p = _pass(da, x, y, acc, part, mode, e=e if ee else None, div=4.0, packed=packed)
                _ffi.check(lib.lgcn_spmm_pass(ctypes.byref(p), N, d, 3, _ffi.stream_of(gpu)), "pass")
            torch.cuda.synchronize()
            outs.append((acc.cpu(), y.cpu()))
        for got in outs[1:]:
            assert torch.equal(got[0], outs[0][0]) and torch.equal(got[1], outs[0][1]), mode


@pytest.mark.parametrize("d", [4, 16, 64, 256, 1024])
def test_spmm_pass_small_row_combine_outside_contract(gpu, d):
    """every split row handed to the one-per-lane-group combine (n_split_big = 0,
    with hub rows of hundreds of chunks among them, no pack_split_rows) is still combined in
    combine_row's association — bitwise lgcn_spmm's rows."""
    import graphs

    from lgcn_amd import _ffi
    from lgcn_amd.propagate import spmm

    U, I, ei = graphs.hub(U=1500, I=40, seed=1)
    N = U + I
    da = _direction(gpu, ei, N, 2, U)
    pc = da.splits[:da.n_splits, 2].cpu()
    assert int(pc.max()) > 16 and int(pc.min()) <= 16  # big and small rows both
    g = torch.Generator(device=gpu).manual_seed(d)
    x = torch.randn(N, d, device=gpu, generator=g)
    part = torch.empty((max(1, da.n_partials), d), device=gpu)
    lib = _ffi.load()
    acc0 = torch.full((N, d), 0.5, device=gpu)
    spmm(da, N, d, (x, None, N), None, (acc0, None, N), None, _ffi.EPI_STORE, 1.0, 1.0, part)
    acc1 = torch.full((N, d), 0.5, device=gpu)
    p = _ffi.Pass(da.items.data_ptr(), da.n_items, da.splits.data_ptr(), da.n_splits, da.col.data_ptr(),
                  da.val.data_ptr(), x.data_ptr(), None, N, None, None, N, None, acc1.data_ptr(), None, N,
                  part.data_ptr(), _ffi.EPI_STORE, 1.0, 1.0, n_split_big=0)
    _ffi.check(lib.lgcn_spmm_pass(ctypes.byref(p), N, d, 3, _ffi.stream_of(gpu)), "pass")
    torch.cuda.synchronize()
    assert torch.equal(acc0.cpu(), acc1.cpu())
