"""The parity bar of SURVEY.md §8c, shared by every HIP-vs-oracle test.

Per row r of an [rows, d] result: ``max|y[r] - ref[r]| <= RTOL * max|ref[r]|`` (a row whose
reference is all zero must be exactly zero). Every check also reports the largest elementwise
relative error over the entries with ``|ref| > 1e-6``. Rows are judged one by one, so small
rows (low-degree, degree-0) are held to their own scale, not to the table's largest value.
"""
from __future__ import annotations

import numpy as np

RTOL = 1e-5  # BASELINE.json north_star: 1e-5 relative fp32


def _2d(a):
    a = np.asarray(a, np.float64)
    if a.ndim == 1:
        return a.reshape(-1, 1)
    return a.reshape(a.shape[0], -1)


def row_errors(y, ref):
    """(max row-relative error, max elementwise relative error where |ref| > 1e-6, index of the
    worst row). Rows whose reference is all zero count as error inf unless y is zero there too."""
    y, ref = _2d(y), _2d(ref)
    if y.shape != ref.shape:
        raise AssertionError(f"shape mismatch {y.shape} vs {ref.shape}")
    if ref.size == 0:
        return 0.0, 0.0, -1
    diff = np.abs(y - ref)
    err = diff.max(axis=1)
    scale = np.abs(ref).max(axis=1)
    with np.errstate(divide="ignore", invalid="ignore"):
        rr = np.where(scale > 0, err / np.where(scale > 0, scale, 1.0), np.where(err > 0, np.inf, 0.0))
    big = np.abs(ref) > 1e-6
    elem = float((diff[big] / np.abs(ref[big])).max()) if big.any() else 0.0
    worst = int(rr.argmax())
    return float(rr[worst]), elem, worst


def assert_rows_close(y, ref, rtol: float = RTOL, what: str = "") -> tuple[float, float]:
    rr, elem, worst = row_errors(y, ref)
    if not rr <= rtol:
        raise AssertionError(f"{what}: row {worst} off by {rr:.3g} of its max |ref| (bar {rtol:g}); "
                             f"max elementwise rel err (|ref| > 1e-6) {elem:.3g}")
    return rr, elem
