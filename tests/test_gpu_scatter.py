"""The per-step negatives scatter (lgcn_range_scatter_add + lgcn_flagged_rows_add) against a
sequential CPU restatement: out[off + key[b]] += (Σ_b in b order C[b]) * mul / div, and the
parked second-source sums Σ_b C2[b] per row. Bit-exact for in-capacity inputs (same b-order
fp32 sums, mul-then-div), and the overflow flag for concentrated keys."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref_scatter(keys, C, out, off, mul, div):
    out = out.copy()
    rows = {}
    for b, k in enumerate(keys):  # first-occurrence order does not matter; per-row order is b order
        rows.setdefault(int(k), []).append(b)
    sums = {}
    for k, bs in rows.items():
        acc = np.zeros(C.shape[1], np.float32)
        for b in bs:
            acc = (acc + C[b]).astype(np.float32)
        sums[k] = acc
        out[off + k] = out[off + k] + (acc * np.float32(mul)) / np.float32(div)
    return out, rows


def _run(gpu, keys_np, nrows, off, d, N, mul, div, with_c2=True, seed=0, sorted_=False, store_unless=None):
    from lgcn_amd import _ffi

    lib = _ffi.load()
    rng = np.random.default_rng(seed)
    B = keys_np.size
    C = rng.standard_normal((B, d)).astype(np.float32)
    C2 = rng.standard_normal((B, d)).astype(np.float32)
    out0 = rng.standard_normal((N, d)).astype(np.float32)
    split = off + nrows // 2  # two tables, split inside the key range
    lo = torch.from_numpy(out0[:split].copy()).to(gpu)
    hi = torch.from_numpy(out0[split:].copy()).to(gpu)
    keys = torch.from_numpy(keys_np.astype(np.int64)).to(gpu)
    Cg, C2g = torch.from_numpy(C).to(gpu), torch.from_numpy(C2).to(gpu)
    buf = torch.empty((max(B, 1), d), dtype=torch.float32, device=gpu)
    flag = torch.empty(max(B, 1), dtype=torch.uint8, device=gpu)
    ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
    s = _ffi.stream_of(gpu)
    su = None if store_unless is None else torch.from_numpy(store_unless).to(gpu)
    if sorted_:  # one stable radix sort of the keys, then one lane group per row
        rowptr = torch.empty(nrows + 1, dtype=torch.int64, device=gpu)
        col = torch.empty(max(B, 1), dtype=torch.int32, device=gpu)
        perm = torch.empty(max(B, 1), dtype=torch.int32, device=gpu)
        err = torch.zeros(1, dtype=torch.int64, device=gpu)
        nb = _ffi._sz(0)
        _ffi.check(lib.lgcn_csr_workspace_size(B, nrows, nb), "ws")
        ws = torch.empty(max(1, nb.value), dtype=torch.uint8, device=gpu)
        _ffi.check(lib.lgcn_csr_build(keys.data_ptr(), keys.data_ptr(), B, nrows, rowptr.data_ptr(), col.data_ptr(),
                                      perm.data_ptr(), err.data_ptr(), ws.data_ptr(), ws.numel(), s), "csr")
        _ffi.check(lib.lgcn_sorted_scatter_add(rowptr.data_ptr(), perm.data_ptr(), nrows, off, Cg.data_ptr(), d,
                                               lo.data_ptr(), hi.data_ptr(), split, mul, div,
                                               C2g.data_ptr() if with_c2 else None, None, None, 0, 0.0, 0,
                                               buf.data_ptr(), flag.data_ptr(), _ffi.ptr(su), s),
                   "lgcn_sorted_scatter_add")
        assert int(err.item()) == 0
    else:
        _ffi.check(lib.lgcn_range_scatter_add(keys.data_ptr(), B, nrows, off, Cg.data_ptr(), d, lo.data_ptr(),
                                              hi.data_ptr(), split, mul, div,
                                              C2g.data_ptr() if with_c2 else None, None, None, 0, 0.0, 0,
                                              buf.data_ptr(), flag.data_ptr(), ovf.data_ptr(), _ffi.ptr(su), s),
                   "lgcn_range_scatter_add")
    after1 = torch.cat([lo, hi]).cpu().numpy()
    if with_c2:
        _ffi.check(lib.lgcn_flagged_rows_add(keys.data_ptr(), B, off, buf.data_ptr(), flag.data_ptr(), d,
                                             lo.data_ptr(), hi.data_ptr(), split, s), "lgcn_flagged_rows_add")
    after2 = torch.cat([lo, hi]).cpu().numpy()
    return C, C2, out0, after1, after2, int(ovf.item()), flag.cpu().numpy()[:B]


@pytest.mark.parametrize("B,nrows,d", [(1, 7, 64), (1000, 500, 64), (10000, 59047, 128), (30000, 5000, 64),
                                       (4000, 300000, 32), (2000, 1000, 256)])
def test_range_scatter_matches_sequential(gpu, B, nrows, d):
    rng = np.random.default_rng(B + nrows)
    keys = rng.integers(0, nrows, B)
    off = 11
    N = off + nrows + 3
    mul, div = float(np.float32(1 / 4)), 4.0
    C, C2, out0, after1, after2, ovf, flag = _run(gpu, keys, nrows, off, d, N, mul, div)
    assert ovf == 0
    ref1, rows = _ref_scatter(keys, C, out0, off, mul, div)
    np.testing.assert_array_equal(after1, ref1)
    ref2, _ = _ref_scatter(keys, C2, ref1, off, 1.0, 1.0)
    np.testing.assert_array_equal(after2, ref2)
    # exactly one flagged slot per distinct row: its first occurrence
    firsts = sorted(bs[0] for bs in rows.values())
    np.testing.assert_array_equal(np.nonzero(flag)[0], firsts)


@pytest.mark.parametrize("B,nrows,d,bad", [(1000, 500, 64, False), (10000, 59047, 128, True), (30000, 5000, 64, False),
                                           (4000, 300000, 32, True), (3000, 10, 64, False)])
def test_range_scatter_counts(gpu, B, nrows, d, bad):
    """lgcn_range_scatter_add_counts (ABI 10): the same out rows and flags as the sequential
    restatement, reg_count[r] = the number of keys of row r for EVERY row (0 included, the buffer
    starts as garbage), keys outside [0, nrows) flagged 0 and counted nowhere."""
    from lgcn_amd import _ffi

    lib = _ffi.load()
    rng = np.random.default_rng(B + nrows + 1)
    keys_np = rng.integers(0, nrows, B)
    if bad:
        keys_np[::97] = nrows + 3
        keys_np[1::89] = -2
    off = 11
    N = off + nrows + 3
    mul, div = float(np.float32(1 / 4)), 4.0
    C = rng.standard_normal((B, d)).astype(np.float32)
    out0 = rng.standard_normal((N, d)).astype(np.float32)
    split = off + nrows // 2
    lo = torch.from_numpy(out0[:split].copy()).to(gpu)
    hi = torch.from_numpy(out0[split:].copy()).to(gpu)
    keys = torch.from_numpy(keys_np.astype(np.int64)).to(gpu)
    Cg = torch.from_numpy(C).to(gpu)
    flag = torch.full((B,), 7, dtype=torch.uint8, device=gpu)
    cnt = torch.full((nrows,), -5, dtype=torch.int32, device=gpu)
    ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
    s = _ffi.stream_of(gpu)
    _ffi.check(lib.lgcn_range_scatter_add_counts(keys.data_ptr(), B, nrows, off, Cg.data_ptr(), d, lo.data_ptr(),
                                                 hi.data_ptr(), split, mul, div, flag.data_ptr(), ovf.data_ptr(), None,
                                                 cnt.data_ptr(), None, 0, 0, 0.0, None, None, 0.0, s),
               "lgcn_range_scatter_add_counts")
    assert int(ovf.item()) == 0
    inside = (keys_np >= 0) & (keys_np < nrows)
    ref, rows = _ref_scatter(keys_np[inside], C[inside], out0, off, mul, div)
    np.testing.assert_array_equal(torch.cat([lo, hi]).cpu().numpy(), ref)
    np.testing.assert_array_equal(cnt.cpu().numpy(), np.bincount(keys_np[inside], minlength=nrows))
    idx = np.nonzero(inside)[0]
    firsts = sorted(int(idx[bs[0]]) for bs in rows.values())
    np.testing.assert_array_equal(np.nonzero(flag.cpu().numpy())[0], firsts)
    assert set(np.unique(flag.cpu().numpy())) <= {0, 1}


def test_range_scatter_empty_and_single_row(gpu):
    # B = 0 is a no-op
    C, C2, out0, after1, after2, ovf, _ = _run(gpu, np.zeros(0, np.int64), 10, 0, 64, 10, 1.0, 1.0)
    np.testing.assert_array_equal(after2, out0)
    # every key the same row (well inside capacity): one sum in b order
    keys = np.full(3000, 5)
    C, C2, out0, after1, after2, ovf, flag = _run(gpu, keys, 10, 0, 64, 10, 1.0, 3.0)
    assert ovf == 0
    ref1, _ = _ref_scatter(keys, C, out0, 0, 1.0, 3.0)
    np.testing.assert_array_equal(after1, ref1)
    assert flag.sum() == 1 and flag[0] == 1


def test_range_scatter_overflow_is_reported(gpu):
    # > 4096 keys in one workgroup's range: the dF part stays correct (flushed partial sums,
    # within rounding), and the overflow flag tells the caller the parked sums were split
    rng = np.random.default_rng(3)
    keys = rng.integers(0, 4, 9000)
    C, C2, out0, after1, _, ovf, _ = _run(gpu, keys, 100000, 0, 64, 100000, 1.0, 1.0, with_c2=False)
    ref1, _ = _ref_scatter(keys, C, out0, 0, 1.0, 1.0)
    np.testing.assert_allclose(after1, ref1, rtol=1e-5, atol=1e-4)
    assert ovf == 1


@pytest.mark.parametrize("B,nrows,d", [(1, 7, 64), (30000, 5000, 64), (162000, 59047, 128), (4000, 300000, 32),
                                       (2000, 1000, 256), (9000, 4, 64)])
def test_sorted_scatter_bitwise_range_scatter(gpu, B, nrows, d):
    """lgcn_sorted_scatter_add (the large-B path) == the sequential restatement and, where the
    range scatter stays in capacity, its output bitwise: the dF rows, the parked C2 sums, the
    flags; with store_unless, rows it marks 0 are stored, not added to."""
    rng = np.random.default_rng(B + d)
    keys = rng.integers(0, nrows, B)
    off = 5
    N = off + nrows + 2
    mul, div = float(np.float32(1 / 4)), 4.0
    su = (rng.random(N) < 0.5).astype(np.uint8)
    for store_unless in (None, su):
        C, C2, out0, after1, after2, _, flag = _run(gpu, keys, nrows, off, d, N, mul, div, seed=1, sorted_=True,
                                                     store_unless=store_unless)
        base = out0.copy()
        if store_unless is not None:
            base[store_unless == 0] = 0.0  # stored rows: (0 + v) == v exactly
        ref1, rows = _ref_scatter(keys, C, base, off, mul, div)
        touched = np.zeros(N, bool)
        touched[off + np.unique(keys)] = True
        want1 = np.where(touched[:, None], ref1, out0)
        np.testing.assert_array_equal(after1, want1)
        ref2, _ = _ref_scatter(keys, C2, want1, off, 1.0, 1.0)
        np.testing.assert_array_equal(after2, ref2)
        firsts = sorted(bs[0] for bs in rows.values())
        np.testing.assert_array_equal(np.nonzero(flag)[0], firsts)
        if B <= 4096 * 8 and store_unless is None and len(np.unique(keys)) > 4:
            _, _, _, r1, r2, ovf, rflag = _run(gpu, keys, nrows, off, d, N, mul, div, seed=1)
            if ovf == 0:
                np.testing.assert_array_equal(after1, r1)
                np.testing.assert_array_equal(after2, r2)
                np.testing.assert_array_equal(flag, rflag)


def _kreg(coeff, B, d):
    # k_bpr_fused's float expression: coeff * 2.0f / (float(B) * float(d))
    return np.float32(np.float32(coeff) * np.float32(2.0)) / (np.float32(B) * np.float32(d))


@pytest.mark.parametrize("sorted_", [False, True])
@pytest.mark.parametrize("B,nrows,d", [(3000, 500, 64), (20000, 59047, 128), (5000, 40, 32)])
def test_reg_source_equals_materialised_reg_rows(gpu, sorted_, B, nrows, d):
    """The scatters' reg source (every occurrence of row r contributes kreg * W[r], formed on the
    fly) parks bitwise the sums a materialised C2 = kreg * W[key] table gives (same values in the
    same order), range and sorted paths; lgcn_reg_rows_add == n copies added in sequence."""
    from lgcn_amd import _ffi

    lib = _ffi.load()
    rng = np.random.default_rng(B + d)
    keys_np = rng.integers(0, nrows, B)
    off = 7
    N = off + nrows + 1
    W = (rng.standard_normal((N, d)) * 0.1).astype(np.float32)
    coeff = 5e-3
    kreg = _kreg(coeff, B, d)
    C2 = (kreg * W[off + keys_np]).astype(np.float32)
    s = _ffi.stream_of(gpu)
    keys = torch.from_numpy(keys_np.astype(np.int64)).to(gpu)
    C = torch.from_numpy(rng.standard_normal((B, d)).astype(np.float32)).to(gpu)
    Wg = torch.from_numpy(W).to(gpu)
    split = off + nrows // 2
    res = []
    for mode in ("table", "reg"):
        out = torch.zeros((N, d), device=gpu)
        buf = torch.zeros((B, d), device=gpu)
        flag = torch.zeros(B, dtype=torch.uint8, device=gpu)
        c2 = torch.from_numpy(C2).to(gpu) if mode == "table" else None
        reg = (None, Wg[:split].data_ptr(), Wg[split:].data_ptr(), split, coeff, B) if mode == "reg" else \
              (c2.data_ptr(), None, None, 0, 0.0, 0)
        if sorted_:
            rowptr = torch.empty(nrows + 1, dtype=torch.int64, device=gpu)
            col = torch.empty(B, dtype=torch.int32, device=gpu)
            perm = torch.empty(B, dtype=torch.int32, device=gpu)
            err = torch.zeros(1, dtype=torch.int64, device=gpu)
            nb = _ffi._sz(0)
            _ffi.check(lib.lgcn_csr_workspace_size(B, nrows, nb), "ws")
            ws = torch.empty(max(1, nb.value), dtype=torch.uint8, device=gpu)
            _ffi.check(lib.lgcn_csr_build(keys.data_ptr(), keys.data_ptr(), B, nrows, rowptr.data_ptr(),
                                          col.data_ptr(), perm.data_ptr(), err.data_ptr(), ws.data_ptr(), ws.numel(),
                                          s), "csr")
            _ffi.check(lib.lgcn_sorted_scatter_add(rowptr.data_ptr(), perm.data_ptr(), nrows, off, C.data_ptr(), d,
                                                   out[:split].data_ptr(), out[split:].data_ptr(), split, 1.0, 1.0,
                                                   *reg, buf.data_ptr(), flag.data_ptr(), None, s), "sorted")
        else:
            ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
            _ffi.check(lib.lgcn_range_scatter_add(keys.data_ptr(), B, nrows, off, C.data_ptr(), d,
                                                  out[:split].data_ptr(), out[split:].data_ptr(), split, 1.0, 1.0,
                                                  *reg, buf.data_ptr(), flag.data_ptr(), ovf.data_ptr(), None, s),
                       "range")
            assert int(ovf.item()) == 0
        res.append((out.cpu(), buf.cpu(), flag.cpu()))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][2], res[1][2])
    fl = res[0][2].bool()
    assert torch.equal(res[0][1][fl], res[1][1][fl])
    # lgcn_reg_rows_add over the keys' CSR: n copies of kreg * W[r], added in sequence
    counts = np.bincount(keys_np, minlength=nrows)
    rowptr = torch.zeros(N + 1, dtype=torch.int64)
    rowptr[off + 1:off + nrows + 1] = torch.from_numpy(np.cumsum(counts))
    rowptr[off + nrows + 1:] = int(counts.sum())
    out = torch.from_numpy(W).to(gpu).clone()
    _ffi.check(lib.lgcn_reg_rows_add(rowptr.to(gpu).data_ptr(), None, N, Wg[:split].data_ptr(), Wg[split:].data_ptr(),
                                     split, d, coeff, B, out[:split].data_ptr(), out[split:].data_ptr(), split, s),
               "reg_rows")
    # the same through an explicit row list (every row with contributions, descending order)
    listed = torch.from_numpy((off + np.flatnonzero(counts))[::-1].astype(np.int32).copy()).to(gpu)
    out2 = torch.from_numpy(W).to(gpu).clone()
    _ffi.check(lib.lgcn_reg_rows_add(rowptr.to(gpu).data_ptr(), listed.data_ptr(), listed.numel(), Wg[:split].data_ptr(),
                                     Wg[split:].data_ptr(), split, d, coeff, B, out2[:split].data_ptr(),
                                     out2[split:].data_ptr(), split, s), "reg_rows listed")
    assert torch.equal(out, out2)
    want = W.copy()
    for r in np.flatnonzero(counts):
        v = (kreg * W[off + r]).astype(np.float32)
        acc = np.zeros(d, np.float32)
        for _ in range(counts[r]):
            acc = (acc + v).astype(np.float32)
        want[off + r] = (want[off + r] + acc).astype(np.float32)
    assert np.array_equal(out.cpu().numpy(), want)


def _group_both(gpu, keys_np, R):
    """(rowptr, perm, err) from lgcn_group_keys and from lgcn_csr_build (rowptr, eid, err)."""
    from lgcn_amd import _ffi

    lib = _ffi.load()
    s = _ffi.stream_of(gpu)
    B = keys_np.size
    keys = torch.from_numpy(keys_np.astype(np.int64)).to(gpu)
    out = []
    for how in ("group", "csr"):
        rowptr = torch.full((R + 1,), -7, dtype=torch.int64, device=gpu)
        perm = torch.full((max(B, 1),), -7, dtype=torch.int32, device=gpu)
        err = torch.zeros(1, dtype=torch.int64, device=gpu)
        if how == "group":
            cursor = torch.zeros(int(lib.lgcn_group_keys_cursor_len(R)), dtype=torch.int32, device=gpu)
            for _ in range(2):  # twice: the second call runs on the cursor the first one left
                err.zero_()
                _ffi.check(lib.lgcn_group_keys(keys.data_ptr(), B, R, rowptr.data_ptr(), perm.data_ptr(),
                                               cursor.data_ptr(), err.data_ptr(), s), "lgcn_group_keys")
            assert int(cursor[:R].abs().sum().item()) == 0  # zero on entry, zero again on exit
        else:
            col = torch.empty(max(B, 1), dtype=torch.int32, device=gpu)
            nb = _ffi._sz(0)
            _ffi.check(lib.lgcn_csr_workspace_size(B, R, nb), "ws")
            ws = torch.empty(max(1, nb.value), dtype=torch.uint8, device=gpu)
            _ffi.check(lib.lgcn_csr_build(keys.data_ptr(), keys.data_ptr(), B, R, rowptr.data_ptr(), col.data_ptr(),
                                          perm.data_ptr(), err.data_ptr(), ws.data_ptr(), ws.numel(), s), "csr")
        torch.cuda.synchronize()
        out.append((rowptr.cpu().numpy(), perm.cpu().numpy()[:B], int(err.item())))
    return out


@pytest.mark.parametrize("B,R,dist", [(0, 5, "uniform"), (1, 1, "uniform"), (1000, 7, "uniform"),
                                      (180000, 59047, "uniform"), (162000, 59047, "zipf"), (5000, 100000, "uniform"),
                                      (3000, 10, "one"), (50000, 4097, "uniform")])
def test_group_keys_equals_csr_build(gpu, B, R, dist):
    """lgcn_group_keys (counting sort: atomic count, one-workgroup scan, atomic placement, per-key
    ordering) writes exactly lgcn_csr_build's rowptr and eid: the negatives' grouping of the
    large-B scatter path (planted shape: B ~ 1.8e5 over I = 59,047), skewed keys, one key."""
    rng = np.random.default_rng(B + R)
    if dist == "uniform":
        keys = rng.integers(0, R, B)
    elif dist == "zipf":
        keys = np.minimum(rng.zipf(1.3, B) - 1, R - 1)
    else:
        keys = np.full(B, 3)
    (rp_g, pm_g, e_g), (rp_c, pm_c, e_c) = _group_both(gpu, keys, R)
    np.testing.assert_array_equal(rp_g, rp_c)
    np.testing.assert_array_equal(pm_g, pm_c)
    assert e_g == e_c == 0
    # and what the grouping means: stable order of positions by key
    np.testing.assert_array_equal(pm_g, np.argsort(keys, kind="stable"))
    np.testing.assert_array_equal(rp_g, np.searchsorted(np.sort(keys), np.arange(R + 1)))


def test_group_keys_out_of_range_keys(gpu):
    """Out-of-range keys count in err and are grouped under key 0, as lgcn_csr_build does."""
    keys = np.array([3, -1, 2, 9, 3, 0, 12, 1], dtype=np.int64)
    (rp_g, pm_g, e_g), (rp_c, pm_c, e_c) = _group_both(gpu, keys, 5)
    assert e_g == e_c == 3
    np.testing.assert_array_equal(rp_g, rp_c)
    np.testing.assert_array_equal(pm_g, pm_c)


def test_group_keys_detects_a_dirty_cursor(gpu):
    """Round 2's captured-step fault needed counts that were not zero on entry (the memset node did
    not account for it: tests/test_gpu_memset_capture.py). The grouping now checks what a dirty
    count array breaks — the counts' total against B, every placement and every group against
    perm[0, B) — reports it as err >= 2^32 and writes nothing outside perm (a guard region after it
    stays intact), instead of writing out of bounds."""
    from lgcn_amd import _ffi

    lib = _ffi.load()
    s = _ffi.stream_of(gpu)
    B, R, guard = 20000, 5000, 4096
    keys = torch.from_numpy(np.random.default_rng(1).integers(0, R, B).astype(np.int64)).to(gpu)
    rowptr = torch.empty(R + 1, dtype=torch.int64, device=gpu)
    buf = torch.full((B + guard,), -7, dtype=torch.int32, device=gpu)
    perm = buf[:B]
    err = torch.zeros(1, dtype=torch.int64, device=gpu)
    cursor = torch.zeros(int(lib.lgcn_group_keys_cursor_len(R)), dtype=torch.int32, device=gpu)
    cursor[:R] = 50  # what a skipped reset would leave: large counts everywhere
    _ffi.check(lib.lgcn_group_keys(keys.data_ptr(), B, R, rowptr.data_ptr(), perm.data_ptr(), cursor.data_ptr(),
                                   err.data_ptr(), s), "lgcn_group_keys")
    torch.cuda.synchronize()
    assert int(err.item()) >= 1 << 32
    assert bool((buf[B:] == -7).all().item())
    assert int(cursor[:R].abs().sum().item()) == 0  # left zero for the next call all the same


@pytest.mark.parametrize("B,nrows,d", [(3000, 500, 64), (20000, 59047, 128), (5000, 40, 32), (180000, 59047, 128)])
def test_sorted_no_parking_plus_grouped_reg_equals_parked(gpu, B, nrows, d):
    """The sorted path without the parking table (lgcn_sorted_scatter_add with no second source:
    dF rows + flags, its C rows loaded four at a time) followed by lgcn_grouped_reg_add is bitwise
    the parked path (reg sums parked per row, then lgcn_flagged_rows_add): the same n-copies sums
    added to the same rows; the flags are the same."""
    from lgcn_amd import _ffi

    lib = _ffi.load()
    rng = np.random.default_rng(B + 3 * d)
    keys_np = rng.integers(0, nrows, B)
    off = 9
    N = off + nrows + 1
    W = (rng.standard_normal((N, d)) * 0.1).astype(np.float32)
    coeff = 5e-3
    s = _ffi.stream_of(gpu)
    keys = torch.from_numpy(keys_np.astype(np.int64)).to(gpu)
    C = torch.from_numpy(rng.standard_normal((B, d)).astype(np.float32)).to(gpu)
    Wg = torch.from_numpy(W).to(gpu)
    split = off + nrows // 2
    rowptr = torch.empty(nrows + 1, dtype=torch.int64, device=gpu)
    perm = torch.empty(B, dtype=torch.int32, device=gpu)
    cursor = torch.zeros(int(lib.lgcn_group_keys_cursor_len(nrows)), dtype=torch.int32, device=gpu)
    err = torch.zeros(1, dtype=torch.int64, device=gpu)
    _ffi.check(lib.lgcn_group_keys(keys.data_ptr(), B, nrows, rowptr.data_ptr(), perm.data_ptr(), cursor.data_ptr(),
                                   err.data_ptr(), s), "group")
    res = []
    for park in (True, False):
        out = torch.from_numpy(W * 0.5).to(gpu)
        buf = torch.zeros((B, d), device=gpu)
        flag = torch.full((B,), 7, dtype=torch.uint8, device=gpu)
        reg = (None, Wg[:split].data_ptr(), Wg[split:].data_ptr(), split, coeff, B) if park else \
              (None, None, None, 0, 0.0, 0)
        _ffi.check(lib.lgcn_sorted_scatter_add(rowptr.data_ptr(), perm.data_ptr(), nrows, off, C.data_ptr(), d,
                                               out[:split].data_ptr(), out[split:].data_ptr(), split, 0.25, 4.0,
                                               *reg, buf.data_ptr(), flag.data_ptr(), None, s), "sorted")
        if park:
            _ffi.check(lib.lgcn_flagged_rows_add(keys.data_ptr(), B, off, buf.data_ptr(), flag.data_ptr(), d,
                                                 out[:split].data_ptr(), out[split:].data_ptr(), split, s), "flagged")
        else:
            _ffi.check(lib.lgcn_grouped_reg_add(rowptr.data_ptr(), nrows, off, Wg[:split].data_ptr(),
                                                Wg[split:].data_ptr(), split, d, coeff, B, out[:split].data_ptr(),
                                                out[split:].data_ptr(), split, s), "grouped reg")
        res.append((out.cpu(), flag.cpu()))
    assert torch.equal(res[0][1], res[1][1])
    assert torch.equal(res[0][0], res[1][0])


@pytest.mark.parametrize("B,nrows,d", [(1, 7, 64), (1000, 500, 64), (10000, 59047, 128), (16383, 5000, 32)])
def test_range_scatter_with_loss_workgroup_bitwise(gpu, B, nrows, d):
    """lgcn_range_scatter_add_loss (the step's loss sum as one extra workgroup of the scatter's
    launch) writes the same scatter results and flags as lgcn_range_scatter_add and the same loss,
    bit for bit, as lgcn_bpr_loss's own single-block launch."""
    from lgcn_amd import _ffi

    lib = _ffi.load()
    rng = np.random.default_rng(B + d)
    keys = torch.from_numpy(rng.integers(0, nrows, B).astype(np.int64)).to(gpu)
    C = torch.from_numpy(rng.standard_normal((B, d)).astype(np.float32)).to(gpu)
    C2 = torch.from_numpy(rng.standard_normal((B, d)).astype(np.float32)).to(gpu)
    terms = torch.from_numpy((rng.standard_normal(2 * B) * 3).astype(np.float32)).to(gpu)
    out0 = torch.from_numpy(rng.standard_normal((nrows, d)).astype(np.float32)).to(gpu)
    s = _ffi.stream_of(gpu)
    res = []
    for fused in (False, True):
        out = out0.clone()
        buf = torch.empty((B, d), dtype=torch.float32, device=gpu)
        flag = torch.empty(B, dtype=torch.uint8, device=gpu)
        ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
        loss = torch.full((1,), float("nan"), dtype=torch.float32, device=gpu)
        common = (keys.data_ptr(), B, nrows, 0, C.data_ptr(), d, out.data_ptr(), None, nrows, 0.25, 4.0,
                  C2.data_ptr(), None, None, 0, 0.0, 0, buf.data_ptr(), flag.data_ptr(), ovf.data_ptr(), None)
        if fused:
            _ffi.check(lib.lgcn_range_scatter_add_loss(*common, terms.data_ptr(), B, d, 1e-4, loss.data_ptr(), s),
                       "lgcn_range_scatter_add_loss")
        else:
            _ffi.check(lib.lgcn_range_scatter_add(*common, s), "lgcn_range_scatter_add")
            _ffi.check(lib.lgcn_bpr_loss(terms.data_ptr(), B, d, 1e-4, loss.data_ptr(), None, s), "lgcn_bpr_loss")
        res.append((out.cpu().numpy(), buf.cpu().numpy(), flag.cpu().numpy(), float(loss.item()), int(ovf.item())))
    (o0, b0, f0, l0, v0), (o1, b1, f1, l1, v1) = res
    assert np.array_equal(o0, o1) and np.array_equal(f0, f1) and v0 == v1 == 0
    assert np.array_equal(b0[f0 == 1], b1[f1 == 1])  # parked sums (first-occurrence slots)
    assert np.float32(l0).tobytes() == np.float32(l1).tobytes() and np.isfinite(l1)


def test_range_scatter_loss_rejects_two_stage_sizes(gpu):
    """The fused loss covers only the single-block sums: B >= LGCN_LOSS_FUSED_MAX_B is refused."""
    from lgcn_amd import _ffi

    lib = _ffi.load()
    B = _ffi.LOSS_FUSED_MAX_B
    z = torch.zeros(1, dtype=torch.float32, device=gpu)
    rc = lib.lgcn_range_scatter_add_loss(z.data_ptr(), B, 10, 0, z.data_ptr(), 64, z.data_ptr(), None, 10, 1.0, 1.0,
                                         None, None, None, 0, 0.0, 0, None, None, None, None, z.data_ptr(), B, 64,
                                         0.0, z.data_ptr(), _ffi.stream_of(gpu))
    assert rc == _ffi.E_ARG
