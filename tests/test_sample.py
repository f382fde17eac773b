"""lgcn_legacy_choice (host C++) reproduces numpy's legacy np.random.choice(n, size,
replace=False) — the reference's Recall@k user draw (utils/train_test.py:187) — pick for pick,
and leaves the global generator in the state numpy itself would."""
import numpy as np
import pytest


@pytest.mark.parametrize("n,size,draws", [(1, 1, 3), (2, 1, 5), (100, 100, 2), (1000, 17, 4), (621562, 100, 2),
                                          (70001, 0, 2), (5, 3, 50)])
def test_legacy_choice_matches_numpy(n, size, draws):
    from lgcn_amd.recall import legacy_choice

    for seed in (0, 7, 12345):
        np.random.seed(seed)
        np.random.random(seed % 5)  # start mid-block
        got = legacy_choice(n, size, draws)
        after = np.random.get_state()
        np.random.seed(seed)
        np.random.random(seed % 5)
        want = np.stack([np.random.choice(n, size, replace=False) for _ in range(draws)])
        ref_after = np.random.get_state()
        np.testing.assert_array_equal(got, want)
        assert after[2] == ref_after[2]
        np.testing.assert_array_equal(after[1], ref_after[1])


def test_legacy_choice_errors_like_numpy():
    from lgcn_amd.recall import legacy_choice

    with pytest.raises(ValueError):
        legacy_choice(5, 6, 1)


@pytest.mark.parametrize("threads", [1, 2, 3, 16])
def test_legacy_choice_parallel_draws_match_numpy(tune, threads):
    """The evaluate() shape (10 draws of 100 from 621,562): draws run on worker threads from the
    states the main thread's accept-test walk hands them; any thread count gives numpy's picks
    and numpy's final state."""
    from lgcn_amd.recall import legacy_choice

    tune(choice_threads=threads)
    np.random.seed(11)
    np.random.random(3)
    got = legacy_choice(621562, 100, 10)
    after = np.random.get_state()
    np.random.seed(11)
    np.random.random(3)
    want = np.stack([np.random.choice(621562, 100, replace=False) for _ in range(10)])
    ref_after = np.random.get_state()
    np.testing.assert_array_equal(got, want)
    assert after[2] == ref_after[2]
    np.testing.assert_array_equal(after[1], ref_after[1])
