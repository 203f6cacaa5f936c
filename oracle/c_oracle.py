"""ctypes binding of oracle/liboracle_als.so — TEST INFRASTRUCTURE ONLY.

The C restatement of Spark's packed dspr + dppsv per-row arithmetic
(oracle/als_oracle.c).  Used by tests/ to cross-check the numpy oracle and by
bench.py's cpu_baseline leg (kind "port").  Never imported by the product.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle_als.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C oracle` (or __graft_entry__.build())")
        L = ctypes.CDLL(path)
        P = ctypes.c_void_p
        L.oracle_half_sweep.argtypes = [P, P, P, ctypes.c_int32, P, ctypes.c_int32, ctypes.c_int32,
                                        ctypes.c_double, ctypes.c_int, ctypes.c_double, P, P,
                                        ctypes.c_int32, P, ctypes.c_int]
        L.oracle_half_sweep.restype = ctypes.c_int
        L.oracle_yty.argtypes = [P, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, P, ctypes.c_int]
        L.oracle_yty.restype = ctypes.c_int
        _LIB = L
    return _LIB


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def yty_packed_upper(Y: np.ndarray, threads: int = 0) -> np.ndarray:
    Y = np.ascontiguousarray(Y, dtype=np.float32)
    k = Y.shape[1]
    out = np.zeros(k * (k + 1) // 2)
    lib().oracle_yty(_p(Y), Y.shape[0], k, k, _p(out), threads)
    return out


def half_sweep(indptr, indices, vals, Y, reg, implicit=False, alpha=1.0, threads=0):
    """Returns (X float32 [n_rows, k], status int32 [n_rows])."""
    indptr = np.ascontiguousarray(indptr, dtype=np.int64)
    indices = np.ascontiguousarray(indices, dtype=np.int32)
    vals = np.ascontiguousarray(vals, dtype=np.float32)
    Y = np.ascontiguousarray(Y, dtype=np.float32)
    n_rows = len(indptr) - 1
    k = Y.shape[1]
    X = np.zeros((n_rows, k), dtype=np.float32)
    st = np.zeros(n_rows, dtype=np.int32)
    G = yty_packed_upper(Y, threads) if implicit else np.zeros(1)
    lib().oracle_half_sweep(_p(indptr), _p(indices), _p(vals), n_rows, _p(Y), k, k, float(reg),
                            int(bool(implicit)), float(alpha), _p(G), _p(X), k, _p(st), threads)
    return X, st
