"""The C ABI boundary without a GPU: liblgcn.so loads, exports exactly what include/lgcn.h
declares, the ctypes table covers it, argument errors come back as codes + messages, and the
product path refuses to run without a ROCm device (no silent CPU fallback)."""
import ctypes
import re
import subprocess

import pytest
import torch

from conftest import ROOT

HEADER = ROOT / "include" / "lgcn.h"


def declared_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(lgcn_\w+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("lgcn_csr_build", "lgcn_edge_norm", "lgcn_inv_sqrt_degree",
                 "lgcn_schedule_build", "lgcn_spmm", "lgcn_spmm_items", "lgcn_spmm_combine", "lgcn_scale",
                 "lgcn_partition_edges", "lgcn_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from lgcn_amd import _ffi

    lib = _ffi.load()
    names = declared_functions()
    for n in names:
        assert hasattr(lib, n), n
    assert sorted(_ffi.EXPORTED) == names
    nm = subprocess.run(["nm", "-D", "--defined-only", str(_ffi.LIB_PATH)], capture_output=True, text=True, check=True)
    exported = sorted(set(re.findall(r"\bT (lgcn_\w+)$", nm.stdout, flags=re.M)))
    assert exported == names


def test_abi_version_and_error_codes():
    from lgcn_amd import _ffi

    lib = _ffi.load()
    assert lib.lgcn_abi_version() == _ffi.ABI_VERSION == 11
    b = ctypes.c_size_t(0)
    assert lib.lgcn_csr_workspace_size(-1, 5, ctypes.byref(b)) == -1
    assert b"bad args" in lib.lgcn_last_error()
    assert lib.lgcn_csr_workspace_size(1 << 40, 5, ctypes.byref(b)) == -3
    # lgcn_spmm validates before touching the device
    rc = lib.lgcn_spmm(None, 1, None, 0, None, None, -1, 64, None, None, 0, None, None, 0, None, None, None, 0, None,
                       0, 1.0, 1.0, None)
    assert rc == -1 and b"bad sizes" in lib.lgcn_last_error()
    rc = lib.lgcn_spmm(None, 1, None, 0, None, None, 4, 64, None, None, 0, None, None, 0, None, None, None, 0, None,
                       9, 1.0, 1.0, None)
    assert rc == -1 and b"bad mode" in lib.lgcn_last_error()
    with pytest.raises(_ffi.LgcnError):
        _ffi.check(-1, "probe")


def test_launch_program_entry_points_refuse_nulls():
    """ABI 11's launch programs check their arguments before any HIP call."""
    from lgcn_amd import _ffi

    lib = _ffi.load()
    h = ctypes.c_void_p()
    assert lib.lgcn_program_from_graph(None, ctypes.byref(h)) == _ffi.E_ARG and h.value is None
    assert b"null" in lib.lgcn_last_error()
    assert lib.lgcn_program_run(None, None) == _ffi.E_ARG
    assert lib.lgcn_program_launches(None) == _ffi.E_ARG
    assert lib.lgcn_program_free(None) == 0


def test_product_path_fails_loudly_without_gpu():
    from lgcn_amd import _ffi
    from models.light_gcn import LightGCN

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    model = LightGCN(4, 3, num_layers=2, dim_h=8)
    ei = torch.tensor([[0, 4], [4, 0]])
    with pytest.raises(_ffi.LgcnError, match="ROCm device"):
        model(ei)


def test_missing_library_is_an_error(tmp_path):
    from lgcn_amd import _ffi

    with pytest.raises(_ffi.LgcnError, match="missing"):
        _ffi.load(tmp_path / "liblgcn.so")


def test_state_dict_keys_match_reference():
    """Q12: only the two embedding tables are state."""
    from models.light_gcn import LightGCN

    m = LightGCN(5, 7, num_layers=3, dim_h=16)
    assert list(m.state_dict()) == ["user_embedding.weight", "item_embedding.weight"]
    assert len(m.convs) == 3


def test_initial_weights_match_reference_init():
    """Same init sequence as reference models/light_gcn.py:22-26 under a fixed seed."""
    from models.light_gcn import LightGCN
    from oracle.lgconv_torch import OracleLightGCN

    torch.manual_seed(5)
    a = LightGCN(11, 13, num_layers=2, dim_h=8)
    torch.manual_seed(5)
    b = OracleLightGCN(11, 13, num_layers=2, dim_h=8)
    assert torch.equal(a.user_embedding.weight, b.user_embedding.weight)
    assert torch.equal(a.item_embedding.weight, b.item_embedding.weight)


def test_get_embeddings_semantics():
    from models.light_gcn import LightGCN

    m = LightGCN(5, 7, num_layers=1, dim_h=4)
    u, i = m.get_embeddings(torch.tensor([0, 2]), torch.tensor([1]))
    assert torch.equal(u, m.user_embedding.weight[[0, 2]]) and torch.equal(i, m.item_embedding.weight[[1]])
    assert m.get_embeddings(user_indices=torch.tensor([1]))[1] is None
    assert m.get_embeddings(item_indices=torch.tensor([1]))[0] is None
    with pytest.warns(UserWarning):
        assert m.get_embeddings() == (None, None)


def test_library_was_built_from_these_sources(monkeypatch):
    """Build provenance: the library carries the sha256 of the sources it was compiled from, and
    the loader refuses a library built from other sources (so GPU runs exercise a binary that
    matches the tree next to it, whoever built it)."""
    from lgcn_amd import _ffi

    assert _ffi.built_sha256() == _ffi.source_sha256() == _ffi.load().lgcn_source_sha256().decode()
    monkeypatch.setattr(_ffi, "_lib", None)
    monkeypatch.setattr(_ffi, "source_sha256", lambda: "0" * 64)
    with pytest.raises(_ffi.LgcnError, match="built from other sources"):
        _ffi.load()


def test_tuning_struct_defaults_validation_and_python_record():
    """ABI 7: the A/B knobs are one process-wide lgcn_tuning_t (no environment reads): defaults are
    the measured choices, lgcn_set_tuning refuses an out-of-range struct and changes nothing, and
    lgcn_amd.tuning carries its native fields into the library and restores them."""
    import dataclasses

    from lgcn_amd import _ffi, tuning

    lib = _ffi.load()
    t = _ffi.Tuning()
    assert lib.lgcn_tuning_defaults(ctypes.byref(t)) == 0
    assert (t.spmm_tail, t.spmm_index_rounds, t.pair_xcds_a, t.partition_refine_rounds,
            t.partition_cluster_rounds, t.choice_threads) == (-1, 0, 4, 16, 8, 16)
    cur = _ffi.Tuning()
    assert lib.lgcn_get_tuning(ctypes.byref(cur)) == 0 and bytes(cur) == bytes(t)
    for field, bad in (("spmm_tail", 2), ("spmm_index_rounds", 3), ("pair_xcds_a", 8), ("choice_threads", 0)):
        b = _ffi.Tuning.from_buffer_copy(bytes(t))
        setattr(b, field, bad)
        assert lib.lgcn_set_tuning(ctypes.byref(b)) == -1 and field.encode() in lib.lgcn_last_error()
    b = _ffi.Tuning.from_buffer_copy(bytes(t))
    b.reserved[3] = 1
    assert lib.lgcn_set_tuning(ctypes.byref(b)) == -1
    assert lib.lgcn_get_tuning(ctypes.byref(cur)) == 0 and bytes(cur) == bytes(t)  # nothing changed
    assert tuning.get() == tuning.Tuning()
    with tuning.tuned(spmm_index_rounds=8, pair_xcds_a=0, slice_mb=4.0):
        assert lib.lgcn_get_tuning(ctypes.byref(cur)) == 0
        assert (cur.spmm_index_rounds, cur.pair_xcds_a) == (8, 0) and tuning.get().slice_mb == 4.0
    assert lib.lgcn_get_tuning(ctypes.byref(cur)) == 0 and bytes(cur) == bytes(t)
    assert tuning.get() == tuning.Tuning()
    with pytest.raises(TypeError):
        tuning.set_tuning(no_such_knob=1)
    with pytest.raises(ValueError):
        tuning.set_tuning(neg_grouping="bogus")
    with pytest.raises(_ffi.LgcnError):
        tuning.set_tuning(spmm_index_rounds=3)
    assert dataclasses.asdict(tuning.get()) == dataclasses.asdict(tuning.Tuning())


def test_product_path_reads_no_environment():
    """No LGCN_* variable reaches a schedule: the package and the library hold no environment
    reads."""
    import pathlib

    pkg = pathlib.Path(__file__).resolve().parent.parent / "movie-recommender-system-with-gnns_amd"
    for f in list(pkg.rglob("*.py")) + list(pkg.rglob("*.hip")) + list(pkg.rglob("*.cpp")) + list(pkg.rglob("*.h")):
        text = f.read_text()
        assert "os.environ" not in text and "getenv" not in text, f
