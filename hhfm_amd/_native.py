"""Loader of the in-tree native extension (``hhfm_amd/lib``).

The product path has no CPU fallback: if ``_hhfm`` (the pybind11 binding of
``libhhfm.so``) is not built, every scoring call raises ``ImportError``.
Build with ``make`` or ``python -c "import __graft_entry__ as g; g.build()"``.
"""
from __future__ import annotations

import importlib.machinery
import importlib.util
import os
import sysconfig

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
LIBHHFM = os.path.join(LIB_DIR, "libhhfm.so")
_EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
PYMOD = os.path.join(LIB_DIR, "_hhfm" + _EXT)

_mod = None


def native():
    """Return the loaded ``_hhfm`` module (loads ``libhhfm.so`` via rpath)."""
    global _mod
    if _mod is None:
        if not os.path.exists(PYMOD):
            raise ImportError(
                f"hhfm_amd native extension missing ({PYMOD}); build it with "
                "`make` (hipcc --offload-arch=gfx950). There is no CPU fallback.")
        loader = importlib.machinery.ExtensionFileLoader("_hhfm", PYMOD)
        spec = importlib.util.spec_from_file_location("_hhfm", PYMOD, loader=loader)
        mod = importlib.util.module_from_spec(spec)
        loader.exec_module(mod)
        _mod = mod
    return _mod
