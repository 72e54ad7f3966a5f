"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY
(checker and bench.py cpu_baseline leg; see cpu_oracle.c for the citations)."""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")
_lib = None

_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            raise ImportError(f"{_LIB} missing: run `make oracle`")
        L = ctypes.CDLL(_LIB)
        L.oracle_fm_out.argtypes = [_i32p, ctypes.c_int64, ctypes.c_int, _f32p, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.c_float, _f32p, ctypes.c_int]
        L.oracle_hhfm_rows.argtypes = [_i32p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p,
                                       ctypes.c_int, _f32p, ctypes.c_int]
        L.oracle_catalog_topk.argtypes = [_i32p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          _f32p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.c_int32, ctypes.c_int, _f32p, _i32p, ctypes.c_int]
        L.oracle_max_threads.restype = ctypes.c_int
        _lib = L
    return _lib


def max_threads() -> int:
    return lib().oracle_max_threads()


def fm_out(X, E, w, w0=0.0, threads=0):
    X = np.ascontiguousarray(X, np.int32)
    E = np.ascontiguousarray(E, np.float32)
    out = np.empty(X.shape[0], np.float32)
    wp = None if w is None else np.ascontiguousarray(w, np.float32).reshape(-1)
    lib().oracle_fm_out(X, X.shape[0], X.shape[1], E, E.shape[1],
                        None if wp is None else wp.ctypes.data, float(w0), out, threads)
    return out


def hhfm_rows(X, E, ctx=(0, 0), time=(0, 0), threads=0):
    X = np.ascontiguousarray(X, np.int32)
    E = np.ascontiguousarray(E, np.float32)
    out = np.empty(X.shape[0], np.float32)
    lib().oracle_hhfm_rows(X, X.shape[0], X.shape[1], ctx[0], ctx[1], time[0], time[1],
                           E, E.shape[1], out, threads)
    return out


def catalog_topk(A, E, mode, K, item_begin, N, w=None, ctx=(0, 0), time=(0, 0), threads=0):
    A = np.ascontiguousarray(A, np.int32)
    E = np.ascontiguousarray(E, np.float32)
    B = A.shape[0]
    s = np.empty((B, K), np.float32)
    i = np.empty((B, K), np.int32)
    wp = None if w is None else np.ascontiguousarray(w, np.float32).reshape(-1)
    rc = lib().oracle_catalog_topk(A, B, A.shape[1], mode, ctx[0], ctx[1], time[0], time[1],
                                   E, E.shape[1], None if wp is None else wp.ctypes.data,
                                   item_begin, N, K, s, i, threads)
    if rc:
        raise ValueError("oracle_catalog_topk: bad K")
    return s, i
