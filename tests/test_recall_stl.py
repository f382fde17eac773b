"""oracle/topk_cpu.py — the libstdc++ selection CPU torch.topk runs (ATen topk_impl_loop) — pinned
against torch.topk itself on tie-heavy rows (CPU; the same function the reference calls at
utils/train_test.py:197 when it runs on a CPU). lgcn_select_topk_stl (csrc/lgcn_recall.hip) runs
these steps on the GPU; tests/test_gpu_recall.py holds it to this module bit for bit."""
import numpy as np
import pytest
import torch

from oracle import topk_cpu


def _tied_rows(rng, rows, M, levels):
    return (rng.integers(0, levels, (rows, M)).astype(np.float32) / levels).astype(np.float32)


@pytest.mark.parametrize("M,k", [(5, 1), (5, 5), (17, 4), (300, 4), (300, 5), (1279, 20), (1280, 20),
                                 (2500, 20), (2500, 100), (6400, 100), (6399, 100), (9000, 100)])
def test_topk_set_matches_torch_cpu_on_ties(M, k):
    """Both of topk_impl_loop's paths (partial_sort from k * 64 <= M, nth_element below) and the
    boundary between them, on rows where most scores tie with others."""
    rng = np.random.default_rng(M * 131 + k)
    for levels in (2, 7, max(2, M // 8), M):
        s = _tied_rows(rng, 6, M, levels)
        _, idx = torch.topk(torch.from_numpy(s), k, dim=1)
        for r in range(s.shape[0]):
            assert np.array_equal(np.sort(idx[r].numpy()), topk_cpu.topk_indices(s[r], k)), (M, k, levels, r)


def test_topk_set_nan_and_signed_zero():
    """NaN ranks above every number and NaNs tie with each other; -0 and +0 are equal."""
    rng = np.random.default_rng(3)
    for M, k in ((40, 7), (700, 9), (3000, 30)):
        s = _tied_rows(rng, 8, M, 5) - np.float32(0.4)
        s[:, rng.integers(0, M, M // 10)] = np.nan
        z = rng.integers(0, M, M // 5)
        s[:, z[: len(z) // 2]] = np.float32(0.0)
        s[:, z[len(z) // 2:]] = np.float32(-0.0)
        _, idx = torch.topk(torch.from_numpy(s), k, dim=1)
        for r in range(s.shape[0]):
            assert np.array_equal(np.sort(idx[r].numpy()), topk_cpu.topk_indices(s[r], k)), (M, k, r)


def test_recall_shaped_duplicates_match_torch_cpu():
    """The reference's own setting: normalised candidate rows drawn with repetition from a small
    item table (every score of a repeated row ties exactly), k = 20 (partial_sort at M = 2,500) and
    k = 100 (nth_element), hit counts as the reference counts them."""
    rng = np.random.default_rng(11)
    items = rng.standard_normal((300, 16)).astype(np.float32)
    cand = torch.from_numpy(items[rng.integers(0, 300, 2500)])
    cand = cand / torch.norm(cand, p=2, dim=1, keepdim=True)
    q = torch.from_numpy(rng.standard_normal((40, 16)).astype(np.float32))
    q = q / torch.norm(q, p=2, dim=1, keepdim=True)
    s = torch.mm(q, cand.t())
    P = 1250
    for k in (20, 100):
        _, idx = torch.topk(s, k, dim=1)
        ref = (idx < P).sum(dim=1).numpy()
        assert np.array_equal(topk_cpu.topk_hits(s.numpy(), k, P), ref), k
    # the lowest-index rule (torch.topk on a GPU) differs from it on such rows
    low = np.array([int((np.lexsort((np.arange(2500), -r))[:20] < P).sum()) for r in s.numpy()])
    assert not np.array_equal(low, topk_cpu.topk_hits(s.numpy(), 20, P))
