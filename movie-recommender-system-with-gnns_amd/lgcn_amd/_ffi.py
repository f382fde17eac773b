"""ctypes binding of liblgcn.so (the C ABI in include/lgcn.h).

This is the whole Python↔native boundary: plain pointers (``tensor.data_ptr()``), sizes and
the caller's HIP stream (``torch.cuda.current_stream().cuda_stream``). No torch types cross it.
The product path has no CPU fallback: if the library is missing, or no ROCm device is present,
every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import pathlib

_HERE = pathlib.Path(__file__).resolve().parent
LIB_PATH = _HERE / "liblgcn.so"

EPI_INIT = 0
EPI_ADD = 1
EPI_FINAL_ACC = 2
EPI_FINAL_E = 3
EPI_STORE = 4
EPI_SCALE = 5

E_ARG, E_WORKSPACE, E_UNSUPPORTED = -1, -2, -3  # include/lgcn.h LGCN_E_*

ITEM_BYTES = 16   # lgcn_item_t {int64 beg; int32 len; int32 dst}
SPLIT_BYTES = 16  # lgcn_split_t {int32 row, pbeg, pcnt, pad}
ABI_VERSION = 11  # LGCN_ABI_VERSION of include/lgcn.h this binding speaks
DIGEST_BLOCKS = 1024  # LGCN_DIGEST_BLOCKS

_lib = None

LOSS_PARTS = 256  # include/lgcn.h LGCN_LOSS_PARTS
LOSS_FUSED_MAX_B = 16384  # include/lgcn.h LGCN_LOSS_FUSED_MAX_B
_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32
_f32 = ctypes.c_float
_sz = ctypes.c_size_t

_SIGS = {
    "lgcn_last_error": ([], ctypes.c_char_p),
    "lgcn_abi_version": ([], ctypes.c_int),
    "lgcn_source_sha256": ([], ctypes.c_char_p),
    "lgcn_tuning_defaults": ([_vp], ctypes.c_int),
    "lgcn_set_tuning": ([_vp], ctypes.c_int),
    "lgcn_get_tuning": ([_vp], ctypes.c_int),
    "lgcn_csr_workspace_size": ([_i64, _i64, ctypes.POINTER(_sz)], ctypes.c_int),
    "lgcn_csr_build": ([_vp, _vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _sz, _vp], ctypes.c_int),
    "lgcn_group_keys": ([_vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp], ctypes.c_int),
    "lgcn_group_keys_cursor_len": ([_i64], _i64),
    "lgcn_inv_sqrt_degree": ([_vp, _i64, _vp, _vp], ctypes.c_int),
    "lgcn_edge_norm": ([_vp, _vp, _i64, _i64, _vp, _vp, _vp], ctypes.c_int),
    "lgcn_schedule_workspace_size": ([_i64, _i64, _i32, ctypes.POINTER(_sz)], ctypes.c_int),
    "lgcn_schedule_build": ([_vp, _i64, _i64, _i32, _i64, _vp, _vp, _i64, _vp, _i64, _vp, _vp, _sz, _vp], ctypes.c_int),
    "lgcn_spmm": ([_vp, _i64, _vp, _i64, _vp, _vp, _i64, _i32,
                   _vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _vp, _i64, _vp, _i32, _f32, _f32, _vp],
                  ctypes.c_int),
    "lgcn_spmm_items": ([_vp, _i64, _vp, _i64, _vp, _vp, _i64, _i32,
                         _vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _vp, _i64, _vp, _i32, _f32, _f32, _vp],
                        ctypes.c_int),
    "lgcn_spmm_combine": ([_vp, _i64, _vp, _i64, _vp, _vp, _i64, _i32,
                           _vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _vp, _i64, _vp, _i32, _f32, _f32, _vp],
                          ctypes.c_int),
    "lgcn_spmm_run": ([_vp, _i64, _vp, _i64, _vp, _vp, _i64, _i32,
                       _vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _vp, _i64, _vp, _i32, _f32, _f32, _vp, _vp],
                      ctypes.c_int),
    "lgcn_spmm_run_slices": ([_vp, _vp, _i32, _vp, _vp, _i64, _i32,
                              _vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _vp, _i64, _vp, _i32, _f32, _f32, _vp, _vp],
                             ctypes.c_int),
    "lgcn_spmm_run_slices_ride": ([_vp, _vp, _i32, _vp, _vp, _i64, _i32,
                                   _vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _vp, _i64, _vp, _i32, _f32, _f32, _vp, _vp,
                                   _vp, _i32],
                                  ctypes.c_int),
    "lgcn_spmm_blocksplit": ([_vp, _i64, _vp, _i64, _vp, _vp, _i64, _i32,
                              _vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _vp, _i64, _vp, _i32, _f32, _f32, _vp, _vp],
                             ctypes.c_int),
    "lgcn_spmm_pair": ([_vp, _vp, _i64, _i32, _i32, _vp], ctypes.c_int),
    "lgcn_spmm_pass": ([_vp, _i64, _i32, _i32, _vp], ctypes.c_int),
    "lgcn_stack_mean_rows": ([_vp, _vp, _i32, _i64, _i32, _vp, _f32, _f32, _vp], ctypes.c_int),
    "lgcn_scale": ([_vp, _vp, _i64, _f32, _f32, _vp], ctypes.c_int),
    "lgcn_copy_scale": ([_vp, _vp, _i64, _i64, _i32, _vp, _f32, _f32, _vp], ctypes.c_int),
    "lgcn_bpr_fused": ([_vp, _vp, _i64, _vp, _vp, _i64, _i64, _vp, _vp, _vp, _i64, _i32, _vp, _f32, _f32, _f32, _vp, _vp,
                        _vp, _vp],
                       ctypes.c_int),
    "lgcn_bpr_fused_cols": ([_vp, _vp, _i64, _vp, _vp, _i64, _i64, _vp, _vp, _vp, _i64, _i32, _i32, _vp, _f32, _f32,
                             _f32, _vp, _i32, _vp, _vp, _vp, _vp], ctypes.c_int),
    "lgcn_bpr_loss": ([_vp, _i64, _i32, _f32, _vp, _vp, _vp], ctypes.c_int),
    "lgcn_loss_accumulate": ([_vp, ctypes.c_double, _vp, _vp], ctypes.c_int),
    "lgcn_segment_rows": ([_vp, _vp, _vp, _i64, _i32, _vp, _vp, _i64, _i32, _f32, _f32, _vp], ctypes.c_int),
    "lgcn_range_scatter_add": ([_vp, _i64, _i64, _i64, _vp, _i32, _vp, _vp, _i64, _f32, _f32, _vp, _vp, _vp, _i64,
                                _f32, _i64, _vp, _vp, _vp, _vp, _vp], ctypes.c_int),
    "lgcn_range_scatter_add_loss": ([_vp, _i64, _i64, _i64, _vp, _i32, _vp, _vp, _i64, _f32, _f32, _vp, _vp, _vp,
                                     _i64, _f32, _i64, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _f32, _vp, _vp],
                                    ctypes.c_int),
    "lgcn_range_scatter_add_counts": ([_vp, _i64, _i64, _i64, _vp, _i32, _vp, _vp, _i64, _f32, _f32, _vp, _vp, _vp,
                                       _vp, _vp, _i64, _i32, _f32, _vp, _vp, ctypes.c_double, _vp], ctypes.c_int),
    "lgcn_sorted_scatter_add": ([_vp, _vp, _i64, _i64, _vp, _i32, _vp, _vp, _i64, _f32, _f32, _vp, _vp, _vp, _i64,
                                 _f32, _i64, _vp, _vp, _vp, _vp], ctypes.c_int),
    "lgcn_grouped_reg_add": ([_vp, _i64, _i64, _vp, _vp, _i64, _i32, _f32, _i64, _vp, _vp, _i64, _vp], ctypes.c_int),
    "lgcn_reg_rows_add": ([_vp, _vp, _i64, _vp, _vp, _i64, _i32, _f32, _i64, _vp, _vp, _i64, _vp], ctypes.c_int),
    "lgcn_adam_consts": ([_vp, _i64, _i64, _f32, ctypes.c_double, ctypes.c_double, _vp], ctypes.c_int),
    "lgcn_row_adam": ([_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _i64, _vp, _i64, _i64, _vp, _vp, _i64,
                       _vp, _vp, _vp, _vp, _f32, _f32, _f32, _f32, _vp, _i32, _vp], ctypes.c_int),
    "lgcn_row_adam_reg": ([_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _i64, _vp, _i64, _i64, _vp, _vp,
                           _vp, _vp, _vp, _f32, _f32, _f32, _f32, _vp, _i32, _vp, _vp], ctypes.c_int),
    "lgcn_row_grad_norm_reg": ([_vp, _vp, _i64, _i32, _vp, _i64, _vp, _i64, _i64, _vp, _vp, _f32, _vp, _vp, _vp, _vp,
                                _vp], ctypes.c_int),
    "lgcn_row_grad_norm_workspace_floats": ([], ctypes.c_int),
    "lgcn_row_grad_norm": ([_vp, _vp, _i64, _i32, _vp, _i64, _vp, _i64, _i64, _vp, _vp, _f32, _vp, _vp, _vp, _vp],
                           ctypes.c_int),
    "lgcn_row_grad_sqnorm": ([_vp, _vp, _i64, _i32, _vp, _i64, _vp, _i64, _i64, _vp, _vp, _vp, _vp], ctypes.c_int),
    "lgcn_row_grad_norm_finish": ([_vp, _i64, _f32, _vp, _vp, _vp], ctypes.c_int),
    "lgcn_owner_reset": ([_vp, _i64, _i64, _i64, _i64, _i64, _vp, _vp], ctypes.c_int),
    "lgcn_owner_pack_rows": ([_vp, _vp, _i64, _i32, _vp, _i64, _vp, _i64, _i64, _vp, _vp, _i64, _i64, _i64, _vp, _vp,
                              _vp, _vp], ctypes.c_int),
    "lgcn_owner_pack_requests": ([_vp, _i64, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _i32,
                                  _vp],
                                 ctypes.c_int),
    "lgcn_rows_gather": ([_vp, _vp, _i64, _i32, _vp, _i64, _vp, _i32, _vp], ctypes.c_int),
    "lgcn_rows_mark": ([_vp, _vp, _i64, _vp, _i32, _vp], ctypes.c_int),
    "lgcn_rows_pack": ([_vp, _vp, _i64, _i32, _vp, _i64, _vp, _i64, _i64, _vp, _vp, _i64, _vp, _vp, _vp],
                       ctypes.c_int),
    "lgcn_rows_mark_first": ([_vp, _i64, _vp, _vp, _vp], ctypes.c_int),
    "lgcn_rows_accumulate": ([_vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _i64, _i32, _f32, _vp], ctypes.c_int),
    "lgcn_recall_width": ([_i32, _vp, _vp], ctypes.c_int),
    "lgcn_normalize_rows": ([_vp, _vp, _i64, _i64, _i32, _vp, _i32, _i64, _vp], ctypes.c_int),
    "lgcn_score_filter": ([_vp, _i64, _i64, _vp, _i64, _i64, _i32, _vp, _vp, _vp, _vp, _i32, _vp], ctypes.c_int),
    "lgcn_select_topk": ([_vp, _vp, _vp, _i32, _i32, _i32, _i64, _i64, _i64, _vp, _vp, _vp], ctypes.c_int),
    "lgcn_digest128": ([_vp, _i64, _vp, _i64, _vp, _vp], ctypes.c_int),
    "lgcn_select_topk_stl": ([_vp, _vp, _i64, _i64, _i32, _i64, _i64, _i64, _vp, _vp], ctypes.c_int),
    "lgcn_legacy_choice": ([_vp, _vp, _i64, _i64, _i64, _vp], ctypes.c_int),
    "lgcn_slice_schedule_workspace_size": ([_i64, _i64, _i32, _i32, _vp, _vp], ctypes.c_int),
    "lgcn_slice_schedule_build": ([_vp, _vp, _i64, _i64, _vp, _i32, _i32, _vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp,
                                   _sz, _vp], ctypes.c_int),
    "lgcn_coalesce_workspace_size": ([_i64, _i64, _vp], ctypes.c_int),
    "lgcn_coalesce_undirected": ([_vp, _vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _sz, _vp], ctypes.c_int),
    "lgcn_flagged_rows_add": ([_vp, _i64, _i64, _vp, _vp, _i32, _vp, _vp, _i64, _vp], ctypes.c_int),
    "lgcn_grad_norm_workspace_floats": ([], ctypes.c_int),
    "lgcn_grad_norm": ([_vp, _i32, _f32, _vp, _vp, _vp], ctypes.c_int),
    "lgcn_adam_step": ([_vp, _i32, _f32, _f32, _f32, _f32, _f32, _f32, _vp, _vp, _i32, _vp], ctypes.c_int),
    "lgcn_adam_prologue": ([_vp, _f32, ctypes.c_double, ctypes.c_double, _vp, _vp], ctypes.c_int),
    "lgcn_program_from_graph": ([_vp, ctypes.POINTER(_vp)], ctypes.c_int),
    "lgcn_program_launches": ([_vp], ctypes.c_int),
    "lgcn_program_run": ([_vp, _vp], ctypes.c_int),
    "lgcn_program_free": ([_vp], ctypes.c_int),
    "lgcn_partition_edges": ([_vp, _vp, _i64, _i64, _i32, _i32, _f32, _vp], ctypes.c_int),
    "lgcn_partition_last_error": ([], ctypes.c_char_p),
}

EXPORTED = tuple(_SIGS)


class AdamTensor(ctypes.Structure):
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
                ("exp_avg_sq", ctypes.c_void_p), ("numel", ctypes.c_int64)]


class Pass(ctypes.Structure):
    """lgcn_pass_t: one lgcn_spmm pass's arguments (lgcn_spmm_pair, lgcn_spmm_pass)."""
    _fields_ = [("items", ctypes.c_void_p), ("n_items", ctypes.c_int64), ("splits", ctypes.c_void_p),
                ("n_splits", ctypes.c_int64), ("col", ctypes.c_void_p), ("val", ctypes.c_void_p),
                ("x_lo", ctypes.c_void_p), ("x_hi", ctypes.c_void_p), ("x_split", ctypes.c_int64),
                ("e_lo", ctypes.c_void_p), ("e_hi", ctypes.c_void_p), ("e_split", ctypes.c_int64),
                ("y", ctypes.c_void_p), ("acc_lo", ctypes.c_void_p), ("acc_hi", ctypes.c_void_p),
                ("acc_split", ctypes.c_int64), ("partial", ctypes.c_void_p), ("mode", ctypes.c_int32),
                ("div", ctypes.c_float), ("mul", ctypes.c_float), ("n_split_big", ctypes.c_int64)]

    def __init__(self, *args, n_split_big: int = -1, **kw):
        super().__init__(*args, **kw)
        self.n_split_big = n_split_big


class Tuning(ctypes.Structure):
    """lgcn_tuning_t (include/lgcn.h, ABI 7)."""
    _fields_ = [("spmm_tail", ctypes.c_int32), ("spmm_index_rounds", ctypes.c_int32),
                ("pair_xcds_a", ctypes.c_int32), ("partition_refine_rounds", ctypes.c_int32),
                ("partition_cluster_rounds", ctypes.c_int32), ("choice_threads", ctypes.c_int32),
                ("reserved", ctypes.c_int32 * 10)]


class RegRows(ctypes.Structure):
    """lgcn_reg_rows_t (include/lgcn.h, ABI 10): a step's reg-gradient rows by occurrence counts."""
    _fields_ = [("w_lo", ctypes.c_void_p), ("w_hi", ctypes.c_void_p), ("w_split", ctypes.c_int64),
                ("coeff", ctypes.c_float), ("B", ctypes.c_int64), ("fixed_rowptr", ctypes.c_void_p),
                ("neg_rowptr", ctypes.c_void_p), ("neg_count", ctypes.c_void_p), ("neg_off", ctypes.c_int64),
                ("neg_rows", ctypes.c_int64)]


class LgcnError(RuntimeError):
    pass


def load(path: os.PathLike | str | None = None) -> ctypes.CDLL:
    """Load liblgcn.so (does not touch the GPU). Raises if it has not been built."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = pathlib.Path(path) if path is not None else LIB_PATH
    if not p.exists():
        raise LgcnError(f"{p} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                        " (the MI355X path has no CPU fallback)")
    lib = ctypes.CDLL(str(p))
    for name, (args, res) in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    if lib.lgcn_abi_version() != ABI_VERSION:
        raise LgcnError(f"liblgcn ABI version {lib.lgcn_abi_version()} != {ABI_VERSION}")
    if path is None:
        built, here = lib.lgcn_source_sha256().decode(), source_sha256()
        if built != here:
            raise LgcnError(f"{p} was built from other sources (sha256 {built[:16]}…) than the tree it is loaded "
                            f"from ({here[:16]}…): rebuild it with __graft_entry__.build()")
        _lib = lib
    return lib


CSRC = _HERE.parent / "csrc"
INCLUDE = _HERE.parent.parent / "include"
# the translation units of liblgcn.so (lgcn_build.cpp carries the hash and is not hashed)
SOURCES = ("lgcn_plan.hip", "lgcn_spmm.hip", "lgcn_optim.hip", "lgcn_bpr.hip", "lgcn_recall.hip", "lgcn_rowadam.hip",
           "lgcn_exchange.hip", "lgcn_partition.cpp", "lgcn_sample.cpp", "lgcn_tuning.cpp", "lgcn_program.cpp")
# the headers they include (csrc/), hashed and tracked as build dependencies with include/lgcn.h
HEADERS = ("lgcn_common.h", "lgcn_exact.h", "lgcn_reg.h")


def source_sha256() -> str:
    """sha256 of the library's sources: each csrc translation unit, the csrc headers, include/lgcn.h
    (name and bytes of each, in that order)."""
    import hashlib

    h = hashlib.sha256()
    for f in [CSRC / s for s in SOURCES + HEADERS] + [INCLUDE / "lgcn.h"]:
        h.update(f.name.encode() + b"\0")
        h.update(f.read_bytes())
    return h.hexdigest()


def built_sha256(path: os.PathLike | str | None = None) -> str | None:
    """The source hash baked into a built library, read from the file (without loading it)."""
    p = pathlib.Path(path) if path is not None else LIB_PATH
    if not p.exists():
        return None
    data = p.read_bytes()
    i = data.find(b"LGCN_SOURCE_SHA256=")
    return data[i + 19:i + 19 + 64].decode() if i >= 0 else None


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().lgcn_last_error().decode(errors="replace")
        raise LgcnError(f"{what} failed (rc={rc}): {msg}")


def ptr(t) -> int | None:
    """data_ptr of a tensor (None for None)."""
    return None if t is None else t.data_ptr()


def require_device(t, what: str) -> None:
    if not t.is_cuda:
        raise LgcnError(f"{what}: the MI355X LightGCN path needs ROCm device tensors, got {t.device}"
                        " (move the model and edge_index to 'cuda'; there is no CPU fallback)")


def stream_of(device) -> int:
    import torch

    return torch.cuda.current_stream(device).cuda_stream
