"""The C-ABI library without a GPU: it loads, exports every symbol declared
in include/hhfm.h, validates arguments before touching the device, and its
host-side pieces (workspace sizing, host top-K merge) are correct."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "hhfm.h")
LIB = os.path.join(ROOT, "hhfm_amd", "lib", "libhhfm.so")


def declared():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(hhfm_\w+)\s*\(", txt, re.M)))


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB)
    names = declared()
    assert len(names) >= 8
    for n in names:
        assert hasattr(lib, n), n
    lib.hhfm_abi_version.restype = ctypes.c_int
    assert lib.hhfm_abi_version() == 1


def test_pybind_module_binds_the_abi():
    from hhfm_amd._native import native
    m = native()
    for n in ["fm_score_rows", "hybrid_score_rows", "catalog_topk", "catalog_topk_workspace",
              "topk_merge", "topk_merge_host"]:
        assert hasattr(m, n)
    assert m.abi_version() == 1


def test_argument_validation_without_device():
    lib = ctypes.CDLL(LIB)
    f = lib.hhfm_fm_score_rows
    f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p,
                  ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                  ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p]
    assert f(None, 0, 5, None, 10, 64, 0, None, 0.0, None, None) == 0        # empty batch
    assert f(None, 10, 5, None, 10, 64, 0, None, 0.0, None, None) == -1      # null ptrs
    assert f(None, 10, 0, None, 10, 64, 0, None, 0.0, None, None) == -1      # F < 1
    assert f(None, 10, 5, None, 10, 64, 7, None, 0.0, None, None) == -1      # dtype
    lib.hhfm_error_string.restype = ctypes.c_char_p
    assert lib.hhfm_error_string(-1) == b"invalid argument"


def test_catalog_argument_errors_raise_valueerror():
    from hhfm_amd._native import native
    m = native()
    with pytest.raises(ValueError):
        m.catalog_topk_workspace(10, 100, 64, 65)     # K > 64
    with pytest.raises(ValueError):                  # K > item_count
        m.catalog_topk(1, 10, 5, 1, 0, 2, 5, 0, 0, 1, 1000, 64, 0, 0, 900, 10, 0, 20,
                       1, 1, 1, 1 << 20, 0)
    with pytest.raises(ValueError):                  # k not a multiple of 8 (fp32)
        m.catalog_topk(1, 10, 5, 1, 0, 2, 5, 0, 0, 16, 1000, 20, 0, 0, 900, 100, 0, 20,
                       1, 1, 1, 1 << 20, 0)
    assert m.catalog_topk_workspace(300, 4082, 64, 20) > 300 * 64 * 4


def test_host_merge_matches_sort():
    from hhfm_amd import ops
    rng = np.random.default_rng(0)
    R, B, K = 5, 50, 20
    sc = rng.integers(0, 6, size=(R, B, K)).astype(np.float32)     # many ties
    ids = np.stack([rng.permutation(1000)[:K] for _ in range(R * B)]).reshape(R, B, K).astype(np.int32)
    order = np.lexsort((ids, -sc), axis=2)
    sc = np.take_along_axis(sc, order, 2)
    ids = np.take_along_axis(ids, order, 2)
    s, i = ops.topk_merge(torch.from_numpy(sc), torch.from_numpy(ids))
    for b in range(B):
        cand = sorted(zip((-sc[:, b]).ravel().tolist(), ids[:, b].ravel().tolist()))[:K]
        assert [c[1] for c in cand] == i[b].tolist()
        assert [-c[0] for c in cand] == s[b].tolist()
