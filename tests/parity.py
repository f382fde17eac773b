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


# ---- the optimizer-trajectory bar (harness / C3 training parity) ------------------------------
# Adam moves a weight by at most about lr per step whatever its gradient, so two runs whose
# gradients differ at the 1e-6 level can disagree in sign on noise-level elements and drift apart
# there by up to ~2 lr per step; those elements ("unsettled": a noise-level gradient, or a first
# moment that nearly cancelled) are exempt from the 1e-5 row bar but are held to that absolute
# bound, and the share of the moved elements that actually leave the row bar is held to
# UNSETTLED_MAX_FRAC. Chosen from the captured runs (profiles/r05d_parity/): at most 7e-5 of the
# moved elements after one step (C3: 45 of 648k user elements, 26 of 1.4M item elements), 0 on the
# golden graph, every one of them within 1e-5 absolute (2 lr = 2e-3 allowed) — bound 1e-3, ~14x.
UNSETTLED_MAX_FRAC = 1e-3


def stats_dir():
    """gpurun_out/parity_stats under the repo root (merged back from the GPU box; copied to
    profiles/ for the record)."""
    import pathlib

    d = pathlib.Path(__file__).resolve().parent.parent / "gpurun_out" / "parity_stats"
    d.mkdir(parents=True, exist_ok=True)
    return d


def record_stats(name: str, stats: dict) -> None:
    import json

    (stats_dir() / f"{name}.json").write_text(json.dumps(stats, indent=1, sort_keys=True, default=float))


def trajectory_bar(got, ref, w0, settled, lr: float, steps: int, what: str,
                   max_frac: float = UNSETTLED_MAX_FRAC, rtol: float = RTOL) -> dict:
    """got / ref / w0: [rows, d] weights after `steps` Adam steps from w0; settled: bool mask of the
    elements held to the per-row rtol bar. Asserts (1) settled elements within rtol of their row's
    scale, (2) every element within 2 lr steps of the reference, (3) the share of the moved
    elements actually outside the rtol row bar (all of them unsettled, by (1)) <= max_frac.
    Returns the counts, including the unsettled (exempted) share the mask allowed."""
    got, ref, w0 = (np.asarray(a, np.float64) for a in (got, ref, w0))
    diff = np.abs(got - ref)
    scale = np.abs(ref).max(axis=1, keepdims=True)
    rel = diff / np.where(scale > 0, scale, 1.0)
    rowrel = float(np.where(settled, rel, 0.0).max()) if ref.size else 0.0
    moved = ref != w0
    n_moved = int(moved.sum())
    unsettled = moved & ~settled
    off_bar = moved & (rel > rtol)
    n_un, n_off = int(unsettled.sum()), int(off_bar.sum())
    frac_off = n_off / max(1, n_moved)
    bound = 2.0 * lr * steps
    max_abs_un = float(diff[unsettled].max()) if n_un else 0.0
    max_abs = float(diff.max()) if diff.size else 0.0
    out = {"settled_row_rel": rowrel, "moved_elements": n_moved, "unsettled_moved": n_un,
           "unsettled_frac": n_un / max(1, n_moved), "off_bar_moved": n_off, "off_bar_frac": frac_off,
           "max_abs_diff_unsettled": max_abs_un, "max_abs_diff": max_abs, "abs_bound_2_lr_steps": bound,
           "steps": steps}
    assert rowrel <= rtol, (what, "settled elements", rowrel)
    assert max_abs <= bound, (what, "|dw| over 2 lr steps", max_abs, bound)
    assert frac_off <= max_frac, (what, "share of moved elements outside the row bar", frac_off, max_frac)
    return out
