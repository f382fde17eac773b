"""ORACLE — test infrastructure, not product code (tests/, __graft_entry__.smoke(), bench.py
cpu_baseline only). ctypes wrapper of oracle/_build/liboracle.so (oracle/lgcn_oracle.c)."""
from __future__ import annotations

import ctypes
import pathlib
import subprocess

import numpy as np

_HERE = pathlib.Path(__file__).resolve().parent
LIB = _HERE / "_build" / "liboracle.so"
_lib = None


def build() -> pathlib.Path:
    subprocess.run(["make", "-s", "-C", str(_HERE)], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        _lib = ctypes.CDLL(str(LIB))
        P = ctypes.c_void_p
        I64, I32 = ctypes.c_int64, ctypes.c_int32
        _lib.oracle_csr_build.argtypes = [P, P, I64, I64, P, P, P]
        _lib.oracle_csr_build.restype = I64
        _lib.oracle_inv_sqrt_degree.argtypes = [P, I64, I64, P]
        _lib.oracle_gcn_norm.argtypes = [P, P, I64, I64, P, P]
        _lib.oracle_lgconv.argtypes = [P, P, P, P, I64, I64, I32, P]
        _lib.oracle_lgconv_transposed.argtypes = [P, P, P, P, I64, I64, I32, P]
        _lib.oracle_lightgcn_forward.argtypes = [P, P, I64, I64, P, P, I64, I32, I32, P, P]
        _lib.oracle_lightgcn_backward.argtypes = [P, I64, P, P, I64, I32, I32, P, P]
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _i64(a):
    return np.ascontiguousarray(a, dtype=np.int64)


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def csr_build(key, other, N: int):
    key, other = _i64(key), _i64(other)
    E = key.size
    rowptr = np.empty(N + 1, np.int64)
    col = np.empty(E, np.int32)
    eid = np.empty(E, np.int32)
    bad = lib().oracle_csr_build(_p(key), _p(other), E, N, _p(rowptr), _p(col), _p(eid))
    if bad:
        raise IndexError(f"{bad} edges out of range")
    return rowptr, col, eid


def gcn_norm(edge_index, N: int):
    src, dst = _i64(edge_index[0]), _i64(edge_index[1])
    dis = np.empty(N, np.float32)
    w = np.empty(src.size, np.float32)
    lib().oracle_gcn_norm(_p(src), _p(dst), src.size, N, _p(dis), _p(w))
    return dis, w


def lgconv(x, edge_index, w):
    x = _f32(x)
    N, d = x.shape
    src, dst, w = _i64(edge_index[0]), _i64(edge_index[1]), _f32(w)
    out = np.empty_like(x)
    lib().oracle_lgconv(_p(x), _p(src), _p(dst), _p(w), src.size, N, d, _p(out))
    return out


def lgconv_transposed(dy, edge_index, w):
    dy = _f32(dy)
    N, d = dy.shape
    src, dst, w = _i64(edge_index[0]), _i64(edge_index[1]), _f32(w)
    out = np.empty_like(dy)
    lib().oracle_lgconv_transposed(_p(dy), _p(src), _p(dst), _p(w), src.size, N, d, _p(out))
    return out


def lightgcn_forward(user_w, item_w, edge_index, K: int):
    uw, iw = _f32(user_w), _f32(item_w)
    U, d = uw.shape
    I = iw.shape[0]
    src, dst = _i64(edge_index[0]), _i64(edge_index[1])
    out = np.empty((U + I, d), np.float32)
    scratch = np.empty((2, U + I, d), np.float32)
    lib().oracle_lightgcn_forward(_p(uw), _p(iw), U, I, _p(src), _p(dst), src.size, d, K, _p(out), _p(scratch))
    return out[:U], out[U:]


def lightgcn_backward(dout, edge_index, U: int, K: int):
    dout = _f32(dout)
    N, d = dout.shape
    src, dst = _i64(edge_index[0]), _i64(edge_index[1])
    grad = np.empty_like(dout)
    scratch = np.empty((2, N, d), np.float32)
    lib().oracle_lightgcn_backward(_p(dout), N, _p(src), _p(dst), src.size, d, K, _p(grad), _p(scratch))
    return grad[:U], grad[U:]
