"""On-device to_undirected / coalesce (lgcn_coalesce_undirected) vs the host coalesce
(torch.unique over row*N+col of both directions — PyG 2.4.0's to_undirected, reference
data/dataset_handler.py:141): bit-exact index arrays."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("U,I,P,seed", [(1, 1, 1, 0), (50, 30, 400, 1), (3000, 800, 60000, 2),
                                        (162541, 59047, 2_000_000, 3)])
def test_coalesce_matches_host(gpu, U, I, P, seed):
    from data.dataset_handler import to_undirected
    from lgcn_amd.ingest import to_undirected as hip

    rng = np.random.default_rng(seed)
    N = U + I
    ei = torch.from_numpy(np.stack([rng.integers(0, U, P), U + rng.integers(0, I, P)]))  # duplicates included
    ref = to_undirected(ei, N)
    got = hip(ei.to(gpu), N).cpu()
    assert torch.equal(got, ref)


def test_coalesce_empty_and_bad_ids(gpu):
    from lgcn_amd.ingest import to_undirected as hip

    out = hip(torch.zeros((2, 0), dtype=torch.int64, device=gpu), 10)
    assert out.shape == (2, 0)
    with pytest.raises(IndexError):
        hip(torch.tensor([[0, 11], [1, 2]], device=gpu), 10)


def test_handler_on_device_matches_host(gpu, tmp_path):
    from data.dataset_handler import MovieLensDataHandler, write_synthetic_movielens

    rp, mp = write_synthetic_movielens(str(tmp_path), 500, 300, 20000, seed=4)
    a = MovieLensDataHandler(rp, mp, device=torch.device("cpu"))
    b = MovieLensDataHandler(rp, mp, device=gpu)
    assert torch.equal(a.edge_index, b.edge_index)
