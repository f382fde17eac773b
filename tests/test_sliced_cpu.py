"""Host logic of the source-sliced schedule (lgcn_amd.sliced), no GPU: the slice boundaries
(slice_bounds: the item range kept whole up to two slices) and the bipartite test that gates the
riding combine (lgcn_spmm_run_slices_ride needs user-table slices to write only item rows and
item-table slices only user rows). Reference: models/light_gcn.py:33 (LGConv per layer)."""
import numpy as np
import torch

from lgcn_amd.plan import slice_bytes_for
from lgcn_amd.sliced import _bipartite, slice_bounds

U_C2, I_C2 = 162_541, 59_047


def test_c2_item_range_is_one_slice_at_d64():
    N = U_C2 + I_C2
    sb = slice_bytes_for(N, 64)
    b = slice_bounds(N, U_C2, 64, sb)
    assert b[0] == 0 and b[-1] == N and U_C2 in b
    assert b.index(U_C2) == len(b) - 2  # one item-table slice
    assert len(b) - 1 == 6  # five 8 MB user-table slices + the item table


def test_item_range_split_beyond_two_slices():
    N = U_C2 + I_C2
    sb = slice_bytes_for(N, 128)  # item table 30 MB > 2 slices of ~13.5 MB
    b = slice_bounds(N, U_C2, 128, sb)
    assert len(b) - 1 - b.index(U_C2) == 3
    assert all(x < y for x, y in zip(b, b[1:]))


def _csr(edges, N):
    src = np.array([e[0] for e in edges], dtype=np.int64)
    dst = np.array([e[1] for e in edges], dtype=np.int64)
    order = np.lexsort((src, dst))
    src, dst = src[order], dst[order]
    rowptr = np.zeros(N + 1, dtype=np.int64)
    np.add.at(rowptr, dst + 1, 1)
    return torch.from_numpy(np.cumsum(rowptr)), torch.from_numpy(src.astype(np.int32))


def test_bipartite_gate():
    U, I = 3, 2
    N = U + I
    both_ways = [(0, 3), (3, 0), (1, 4), (4, 1), (2, 3), (3, 2)]
    assert _bipartite(*_csr(both_ways, N), U)
    assert not _bipartite(*_csr(both_ways + [(0, 1)], N), U)  # user -> user
    assert not _bipartite(*_csr(both_ways + [(3, 4)], N), U)  # item -> item
    assert _bipartite(torch.zeros(N + 1, dtype=torch.int64), torch.zeros(0, dtype=torch.int32), U)
