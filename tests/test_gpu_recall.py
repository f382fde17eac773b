"""Recall@k on the GPU (lgcn_amd.recall, csrc/lgcn_recall.hip) against the CPU restatement
oracle/recall_ref.py (pinned to the reference's own compute_recall_at_k outputs in
tests/test_oracle_recall.py). Hit counts are exact on every query whose k-th and (k+1)-th
float64 scores are separated by more than fp32 rounding; ties take the positives first on both
sides."""
import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import recall_ref as R

pytestmark = pytest.mark.gpu


def _emb(rng, n, d):
    return rng.standard_normal((n, d)).astype(np.float32)


def _check_hits(gpu, users, pos, neg, picked, k, **kw):
    from lgcn_amd.recall import topk_hits

    t = lambda a: torch.from_numpy(a).to(gpu)
    hits = topk_hits(t(users), torch.from_numpy(picked), t(pos), t(neg), k, **kw).cpu().numpy()
    ref, gap = R.topk_hits(users[picked], pos, neg, k, return_gap=True)
    sep = gap > 1e-5
    assert sep.mean() > 0.9
    np.testing.assert_array_equal(hits[sep], ref[sep])
    return hits, ref


@pytest.mark.parametrize("d", [8, 32, 64, 100, 128, 256])
@pytest.mark.parametrize("k", [1, 20, 100])
def test_topk_hits_match_oracle(gpu, d, k):
    rng = np.random.default_rng(d * 1000 + k)
    users, pos, neg = _emb(rng, 900, d), _emb(rng, 3000, d), _emb(rng, 2500, d)
    picked = rng.choice(900, 300, replace=False)
    _check_hits(gpu, users, pos, neg, picked, k)


def test_topk_hits_subset_thresholds_and_overflow(gpu):
    # M = 60k > SUBSET: strided-subset thresholds; then a tiny capacity forces the overflow loop
    rng = np.random.default_rng(5)
    d = 64
    users, pos, neg = _emb(rng, 500, d), _emb(rng, 30000, d), _emb(rng, 30000, d)
    picked = rng.choice(500, 256, replace=False)
    _check_hits(gpu, users, pos, neg, picked, 100)
    _check_hits(gpu, users, pos, neg, picked, 100, cap=512, subset=512)


def test_topk_hits_ties_take_positives_first(gpu):
    # every negative duplicates a positive: each score appears twice, positives first
    rng = np.random.default_rng(6)
    d = 32
    users, pos = _emb(rng, 200, d), _emb(rng, 400, d)
    neg = pos[rng.permutation(400)]
    picked = rng.choice(200, 100, replace=False)
    from lgcn_amd.recall import topk_hits

    t = lambda a: torch.from_numpy(a).to(gpu)
    for k in (1, 7, 20):
        hits = topk_hits(t(users), torch.from_numpy(picked), t(pos), t(neg), k).cpu().numpy()
        np.testing.assert_array_equal(hits, R.topk_hits(users[picked], pos, neg, k))


def test_topk_hits_edge_cases(gpu):
    from lgcn_amd.recall import topk_hits

    rng = np.random.default_rng(7)
    users, pos, neg = _emb(rng, 10, 16), _emb(rng, 3, 16), _emb(rng, 2, 16)
    t = lambda a: torch.from_numpy(a).to(gpu)
    picked = np.arange(10)
    # k == M: every positive is a hit
    hits = topk_hits(t(users), torch.from_numpy(picked), t(pos), t(neg), 5).cpu().numpy()
    np.testing.assert_array_equal(hits, np.full(10, 3))
    with pytest.raises(RuntimeError, match="out of range"):
        topk_hits(t(users), torch.from_numpy(picked), t(pos), t(neg), 6)
    # no negatives at all
    hits = topk_hits(t(users), torch.from_numpy(picked), t(pos), t(neg[:0]), 2).cpu().numpy()
    np.testing.assert_array_equal(hits, np.full(10, 2))


def test_compute_recall_at_k_matches_reference_golden(gpu):
    """The reference's own compute_recall_at_k values (tests/golden/harness.npz, made by
    importing reference utils/train_test.py), reproduced through the HIP path."""
    from utils import train_test as TT

    G = np.load(GOLDEN / "harness.npz")
    embs = tuple(torch.from_numpy(a.copy()).to(gpu) for a in G["recall_embs"])
    for k in (20, 100):
        np.random.seed(7)
        r = TT.compute_recall_at_k(embs, k=k)
        assert r == pytest.approx(float(G[f"recall_k{k}"]), rel=1e-6, abs=0)


def test_compute_recall_at_k_matches_oracle_at_scale(gpu):
    """At 40k x 80k candidates, d=128: every query whose k-th and (k+1)-th float64 scores are
    separated by more than fp32 rounding gets exactly the oracle's hit count; an unseparated query
    (a near-tie at the k-th place, whose order even the reference's torch.topk leaves to rounding)
    may differ by one hit; and compute_recall_at_k equals the reference formula over the HIP
    hit counts to the bit (same picks, same float32 reductions)."""
    from lgcn_amd.recall import topk_hits
    from utils import train_test as TT

    rng = np.random.default_rng(8)
    d = 128
    users, pos, neg = _emb(rng, 40000, d), _emb(rng, 40000, d), _emb(rng, 40000, d)
    np.random.seed(3)
    ref, detail = R.recall_at_k((users, pos, neg), k=100, return_detail=True)
    np.random.seed(3)
    t = lambda a: torch.from_numpy(a).to(gpu)
    got = TT.compute_recall_at_k(tuple(t(a) for a in (users, pos, neg)), k=100)
    unseparated, rows = 0, []
    for picked, hits_ref, gap in detail:
        hits_d = topk_hits(t(users), torch.from_numpy(picked), t(pos), t(neg), 100)
        hits = hits_d.cpu().numpy()
        sep = gap > 1e-5
        np.testing.assert_array_equal(hits[sep], hits_ref[sep])
        assert np.abs(hits[~sep] - hits_ref[~sep]).max(initial=0) <= 1
        unseparated += int((~sep).sum())
        rows.append(hits_d)
    # the reference's per-sample float32 means (hits / P, a 1-D CPU mean per sample), summed in order
    total = 0.0
    for r in rows:
        total += (r.cpu().to(torch.float32) / pos.shape[0]).mean().item()
    assert got == total / len(detail)
    # each unseparated query moves its user's recall by at most 1/P, the result by that / (100 * samples)
    bound = unseparated / (pos.shape[0] * 100 * len(detail))
    assert abs(got - ref) <= bound + 1e-6 * abs(ref)
    print(f"recall@100 {got:.6f} vs oracle {ref:.6f}; unseparated queries {unseparated} of {100 * len(detail)}")


def test_evaluate_overlapped_draws_equal_sequential(gpu):
    """evaluate() on the device starts numpy's Recall user draws on a host thread while the loss
    runs (lgcn_amd.recall.start_picks): same loss, same Recall and same numpy state afterwards as
    the sequential compute_embeddings -> bpr_loss -> compute_recall_at_k."""
    import graphs
    from models.light_gcn import LightGCN
    from utils import train_test as TT

    U, I, ei = graphs.subsampled(U=3000, I=1500, pairs=20000, seed=5)

    class _B:
        edge_index = torch.from_numpy(ei).to(gpu)

        def to(self, _):
            return self

    torch.manual_seed(0)
    model = LightGCN(U, I, num_layers=3, dim_h=64).to(gpu)
    torch.manual_seed(42)
    np.random.seed(43)
    loss_a, rec_a = TT.evaluate(model, _B(), gpu, top_k=100)
    state_a = np.random.get_state()
    torch.manual_seed(42)
    np.random.seed(43)
    with torch.no_grad():
        embs = TT.compute_embeddings(model, _B(), gpu)
        loss_b = TT.bpr_loss(*embs).item()
        rec_b = TT.compute_recall_at_k((embs[1], embs[3], embs[5]), k=100)
    state_b = np.random.get_state()
    assert loss_a == loss_b and rec_a == rec_b
    assert state_a[2] == state_b[2] and np.array_equal(state_a[1], state_b[1])


def _key_scores(keys: np.ndarray) -> np.ndarray:
    """float32 scores from lgcn_score_filter's order-preserving keys (csrc/lgcn_recall.hip key_score)."""
    k = keys.view(np.uint32)
    bits = np.where(k & np.uint32(0x80000000), k ^ np.uint32(0x80000000), ~k).astype(np.uint32)
    return bits.view(np.float32)


def _dup_rows(rng, n_items, d, P, Nn, Q):
    items = _emb(rng, n_items, d)
    return _emb(rng, Q, d), items[rng.integers(0, n_items, P)], items[rng.integers(0, n_items, Nn)]


@pytest.mark.parametrize("P,Nn,k,Q", [(1250, 1250, 20, 200), (1250, 1250, 100, 200), (4500, 4500, 100, 130),
                                      (150, 150, 5, 64), (40000, 40000, 20, 128)])
def test_select_topk_stl_matches_cpu_topk_model(gpu, P, Nn, k, Q):
    """lgcn_select_topk_stl on the GPU's own dense scores == oracle/topk_cpu.py (the libstdc++
    selection CPU torch.topk runs, pinned to torch.topk in tests/test_recall_stl.py) on the same
    scores, query by query: candidate rows repeat (every repeated row's scores tie exactly), and the
    cases cover the partial_sort path (k * 64 <= M: M = 2,500 / k = 20, M = 80,000), the
    nth_element path (M = 2,500 / k = 100, M = 9,000, M = 300) and padded query blocks."""
    from lgcn_amd import _ffi
    from oracle import topk_cpu

    rng = np.random.default_rng(P + k + Q)
    d = 32
    users, pos, neg = _dup_rows(rng, max(8, (P + Nn) // 8), d, P, Nn, Q)
    lib = _ffi.load()
    s = _ffi.stream_of(gpu)
    t = lambda a: torch.from_numpy(a).to(gpu)
    M = P + Nn
    D, Qpad = 32, -(-Q // 128) * 128
    Qn = torch.empty((Qpad, D), dtype=torch.float32, device=gpu)
    Cn = torch.empty((M, D), dtype=torch.float32, device=gpu)
    u, pp, nn_ = t(users), t(pos), t(neg)
    _ffi.check(lib.lgcn_normalize_rows(u.data_ptr(), None, Q, d, d, Qn.data_ptr(), D, Qpad, s), "normalize")
    _ffi.check(lib.lgcn_normalize_rows(pp.data_ptr(), None, P, d, d, Cn.data_ptr(), D, P, s), "normalize")
    _ffi.check(lib.lgcn_normalize_rows(nn_.data_ptr(), None, Nn, d, d, Cn.data_ptr() + P * D * 4, D, Nn, s), "normalize")
    keys = torch.empty((Qpad, M), dtype=torch.int32, device=gpu)
    idx = torch.empty((Qpad, M), dtype=torch.int32, device=gpu)
    _ffi.check(lib.lgcn_score_filter(Qn.data_ptr(), Qpad, Q, Cn.data_ptr(), M, 1, D, None, keys.data_ptr(),
                                     idx.data_ptr(), None, M, s), "lgcn_score_filter")
    scores = _key_scores(keys[:Q].cpu().numpy())
    hits = torch.full((Qpad,), -7, dtype=torch.int32, device=gpu)
    _ffi.check(lib.lgcn_select_topk_stl(keys.data_ptr(), idx.data_ptr(), M, M, k, P, Qpad, Q, hits.data_ptr(), s),
               "lgcn_select_topk_stl")
    got = hits.cpu().numpy()
    assert (got[Q:] == 0).all()
    want = topk_cpu.topk_hits(scores, k, P)
    np.testing.assert_array_equal(got[:Q], want)
    # and the lowest-index rule (lgcn_select_topk) counts differently on these rows
    low = topk_hits_index(gpu, users, pos, neg, k)
    assert (low >= got[:Q]).all() and (low != got[:Q]).any()


def topk_hits_index(gpu, users, pos, neg, k):
    from lgcn_amd.recall import topk_hits

    t = lambda a: torch.from_numpy(a).to(gpu)
    return topk_hits(t(users), torch.arange(users.shape[0]), t(pos), t(neg), k, ties="index").cpu().numpy()


def test_compute_recall_at_k_cpu_ties_equals_reference_on_cpu(gpu, tune):
    """Recall@20 / @100 of duplicate-heavy validation rows (600 items behind 2 x 1,250 candidate
    rows, as a C1 validation batch has them): compute_recall_at_k on device tensors with
    recall_ties="cpu" equals the reference's formula run on the CPU (utils/train_test.py's CPU
    branch: torch.mm + torch.topk), to the bit; the default "index" rule equals the lowest-index
    restatement oracle/recall_ref.py, and the two differ on these rows."""
    from utils import train_test as TT

    rng = np.random.default_rng(21)
    users, pos, neg = _dup_rows(rng, 600, 64, 1250, 1250, 1250)
    host = tuple(torch.from_numpy(a) for a in (users, pos, neg))
    dev = tuple(a.to(gpu) for a in host)
    for k in (20, 100):
        np.random.seed(9)
        ref_cpu = TT.compute_recall_at_k(host, k=k)
        np.random.seed(9)
        tune(recall_ties="cpu")
        got_cpu = TT.compute_recall_at_k(dev, k=k)
        np.random.seed(9)
        tune(recall_ties="index")
        got_index = TT.compute_recall_at_k(dev, k=k)
        np.random.seed(9)
        ref_index = R.recall_at_k((users, pos, neg), k=k)
        print(f"Recall@{k}: cpu ties {got_cpu:.8f} (reference on CPU {ref_cpu:.8f}); "
              f"index ties {got_index:.8f} (oracle {ref_index:.8f})")
        assert got_cpu == ref_cpu, (k, got_cpu, ref_cpu)
        assert got_index == pytest.approx(ref_index, rel=1e-6, abs=0), (k, got_index, ref_index)
        assert got_index != got_cpu


def test_cpu_ties_query_blocks(gpu, tune, monkeypatch):
    """recall_ties="cpu" writes dense score rows per query block (lgcn_amd.recall.STL_BLOCK_BYTES):
    several blocks (the padded queries of the last one included) give the one-block hits."""
    from lgcn_amd import recall as RC

    rng = np.random.default_rng(31)
    users, pos, neg = _dup_rows(rng, 400, 32, 2000, 2000, 700)
    t = lambda a: torch.from_numpy(a).to(gpu)
    picked = torch.from_numpy(rng.choice(700, 600, replace=False))
    for k in (20, 100):  # partial_sort (k * 64 <= 4000) and nth_element
        one = RC.topk_hits(t(users), picked, t(pos), t(neg), k, ties="cpu").cpu()
        monkeypatch.setattr(RC, "STL_BLOCK_BYTES", 8 * 4000 * 128)  # 128 queries per block
        many = RC.topk_hits(t(users), picked, t(pos), t(neg), k, ties="cpu").cpu()
        monkeypatch.setattr(RC, "STL_BLOCK_BYTES", 1 << 30)
        assert torch.equal(one, many), k
