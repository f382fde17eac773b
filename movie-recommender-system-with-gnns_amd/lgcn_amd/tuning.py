"""Process-wide tuning of the path's schedules and kernels (round 5).

Earlier rounds read A/B knobs from environment variables on every dispatch (LGCN_SLICE_MB,
LGCN_SLICE_RIDE, LGCN_SPMM_VARIANT, LGCN_PAIR_XCD, ...), so a stray variable in a user's
environment could silently change a schedule, or a result's last bits. Nothing in the library or
in lgcn_amd reads the environment now: the choices live in one Tuning record, defaulted to the
measured ones, changed only by an explicit call:

    from lgcn_amd import tuning
    tuning.set_tuning(slice_mb=8.0)            # process-wide; returns the previous record
    with tuning.tuned(spmm_index_rounds=2):    # scoped (tests, A/B tools)
        ...

The native fields go to liblgcn.so's lgcn_set_tuning (include/lgcn.h lgcn_tuning_t), the rest
are read by the Python schedule code when it builds or dispatches. Set them before building the
plans they concern (a plan's schedule is built once per width and cached). Knobs whose A/B is
settled were dropped rather than moved here (the 16-deep d = 64 unroll, the
non-temporal override, the block-split switch, the rank chunk).
"""
from __future__ import annotations

import contextlib
import dataclasses

# the fields that live in the library (lgcn_tuning_t)
NATIVE = ("spmm_tail", "spmm_index_rounds", "pair_xcds_a", "partition_refine_rounds",
          "partition_cluster_rounds", "choice_threads")


@dataclasses.dataclass(frozen=True)
class Tuning:
    # --- schedule choices made in Python -------------------------------------------------------
    # source-slice size of full-graph schedules in MiB: None = lgcn_amd.plan.slice_bytes_for's
    # measured choice; 0 = never slice; > 0 = forced (and the density test skipped)
    slice_mb: float | None = None
    # K-layer sliced forward with the split-row combines riding in the next slice group's launch
    slice_ride: bool = True
    # large-batch negatives grouping: "count" (lgcn_group_keys) or "radix" (lgcn_csr_build)
    neg_grouping: str = "count"
    # batch size from which the negatives take the sorted scatter instead of the range scatter
    sorted_scatter_min_b: int = 49152
    # hub chunk (edges per lane-group chain) of a Cluster-GCN batch's propagation plan: None =
    # lgcn_amd.train_step.batch_chunk_for's measured rule (by the batch's edge count); > 0 = forced
    batch_chunk: int | None = None
    # Recall@k: candidates in the strided subset that sets the first thresholds
    recall_subset: int = 16384
    # Recall@k: which of several equal scores make a query's top k (lgcn_amd.recall.topk_hits):
    # "index" — the lowest candidate indices (the positives) first, as torch.topk on a GPU (its
    # gather pass fills the k-th value's ties in index order); "cpu" — exactly what CPU torch.topk
    # keeps (libstdc++ partial_sort / nth_element, lgcn_select_topk_stl)
    recall_ties: str = "index"
    # utils.train_test.train routes eligible calls to the fused batch step (False: reference loop)
    harness_fused: bool = True
    # single-GPU lazy step: the BPR reg-gradient rows formed inside the clip norm and the Adam update
    # from their occurrence counts (lgcn_row_*_reg, bitwise) instead of two passes after the backward
    reg_in_update: bool = True
    # a captured single-GPU training step is issued as a launch program (lgcn_program_run: the
    # graph's kernels launched on the stream from one call, no hipGraphLaunch) instead of replayed
    # as a hipGraph (~8 us of GPU time per replay)
    step_program: bool = True
    # run the exchanges' RCCL branches even on a gloo group (tests: gloo carries the bytes)
    device_collectives: bool = False
    # --- native (lgcn_tuning_t) -----------------------------------------------------------------
    spmm_tail: int = -1
    spmm_index_rounds: int = 0
    pair_xcds_a: int = 4
    partition_refine_rounds: int = 16
    partition_cluster_rounds: int = 8
    choice_threads: int = 16

    def validate(self) -> None:
        if self.slice_mb is not None and not self.slice_mb >= 0:
            raise ValueError(f"slice_mb must be None or >= 0, got {self.slice_mb}")
        if self.neg_grouping not in ("count", "radix"):
            raise ValueError(f"neg_grouping must be 'count' or 'radix', got {self.neg_grouping!r}")
        if self.sorted_scatter_min_b < 1 or self.recall_subset < 1:
            raise ValueError("sorted_scatter_min_b and recall_subset must be >= 1")
        if self.recall_ties not in ("index", "cpu"):
            raise ValueError(f"recall_ties must be 'index' or 'cpu', got {self.recall_ties!r}")
        if self.batch_chunk is not None and self.batch_chunk < 1:
            raise ValueError(f"batch_chunk must be None or >= 1, got {self.batch_chunk}")


_current = Tuning()


def get() -> Tuning:
    return _current


def _apply_native(t: Tuning) -> None:
    from . import _ffi

    lib = _ffi.load()
    rec = _ffi.Tuning()
    _ffi.check(lib.lgcn_tuning_defaults(ctypes_ref(rec)), "lgcn_tuning_defaults")
    for f in NATIVE:
        setattr(rec, f, int(getattr(t, f)))
    _ffi.check(lib.lgcn_set_tuning(ctypes_ref(rec)), "lgcn_set_tuning")


def ctypes_ref(rec):
    import ctypes

    return ctypes.byref(rec)


def set_tuning(**changes) -> Tuning:
    """Replace the named fields (unknown names raise); returns the previous record."""
    global _current
    unknown = set(changes) - {f.name for f in dataclasses.fields(Tuning)}
    if unknown:
        raise TypeError(f"unknown tuning field(s): {sorted(unknown)}")
    new = dataclasses.replace(_current, **changes)
    new.validate()
    if any(getattr(new, f) != getattr(_current, f) for f in NATIVE):  # only a real change loads the library
        _apply_native(new)
    prev, _current = _current, new
    return prev


def reset() -> Tuning:
    """Back to the defaults; returns the previous record."""
    return set_tuning(**dataclasses.asdict(Tuning()))


@contextlib.contextmanager
def tuned(**changes):
    """set_tuning(**changes) for the duration of a with block."""
    prev = set_tuning(**changes)
    try:
        yield _current
    finally:
        set_tuning(**dataclasses.asdict(prev))
