"""Loader for the in-tree HIP kernel library (``csrc/`` -> ``_lib/libddlpc_hip.so``).

The library is built by ``__graft_entry__.build()`` / ``python scripts/build_ext.py`` with
``hipcc --offload-arch=gfx950`` and registers its operators with ``TORCH_LIBRARY(ddlpc)``
so they appear as ``torch.ops.ddlpc.*`` (and by kernel name in rocprof): one op namespace,
two kernels per operator — the gfx950 HIP kernel for GPU tensors and the C++ reference of
``csrc/cpu_ref.cpp`` for CPU tensors, chosen by PyTorch's dispatcher.  Nothing here falls
back silently: requesting the ops without the built library raises.
"""
from __future__ import annotations

import os
import threading

import torch

_LIB_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_lib")
# DDLPC_LIB_PATH: load another build of the same library (A/B of kernel variants)
LIB_PATH = os.environ.get("DDLPC_LIB_PATH") or os.path.join(_LIB_DIR, "libddlpc_hip.so")
_lock = threading.Lock()
_loaded = False
_error = None


def load(strict: bool = True) -> bool:
    global _loaded, _error
    with _lock:
        if _loaded:
            return True
        if not os.path.exists(LIB_PATH):
            _error = f"HIP kernel library not built: {LIB_PATH} (run scripts/build_ext.py)"
        else:
            try:
                torch.ops.load_library(LIB_PATH)
                _loaded = True
                return True
            except Exception as e:       # pragma: no cover - depends on the box
                _error = f"failed to load {LIB_PATH}: {e}"
        if strict:
            raise RuntimeError(_error)
        return False


def available() -> bool:
    return load(strict=False)


def ops():
    """``torch.ops.ddlpc`` — raises if the library is missing (no silent fallback)."""
    load(strict=True)
    return torch.ops.ddlpc


def last_error():
    return _error
