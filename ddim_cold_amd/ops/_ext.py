"""Loader for the in-tree native extension ``ddim_cold_amd/_C.so``.

The extension holds every hand-written gfx950 HIP kernel plus the
``TORCH_LIBRARY(ddim_cold, ...)`` registrations (``csrc/bindings.cpp``).  It is
built in-tree by :mod:`ddim_cold_amd.build` (``hipcc --offload-arch=gfx950``)
so that it travels with the repository snapshot to the GPU box.

Policy: on a GPU tensor the HIP path is mandatory.  If the extension is
missing or fails to load we raise (``NativeExtensionError``) instead of
silently falling back to PyTorch eager ops; set
``DDIM_COLD_ALLOW_REFERENCE=1`` to opt into the slow reference path.
"""
from __future__ import annotations

import os
import threading

import torch

_LOCK = threading.Lock()
_STATE = {"loaded": False, "error": None, "path": None}

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# DDIM_COLD_LIB: load another build of the extension (A/B runs of two builds of
# the same tree, e.g. tools/gpu_lib_ab.sh); default the in-tree _C.so
LIB_PATH = os.environ.get("DDIM_COLD_LIB") or os.path.join(PKG_DIR, "_C.so")


class NativeExtensionError(RuntimeError):
    pass


def load(raise_on_error: bool = False) -> bool:
    with _LOCK:
        if _STATE["loaded"]:
            return True
        if _STATE["error"] is not None and not raise_on_error:
            return False
        if not os.path.isfile(LIB_PATH):
            _STATE["error"] = f"native extension not built: {LIB_PATH} (run python -m ddim_cold_amd.build)"
        else:
            try:
                torch.ops.load_library(LIB_PATH)
                _STATE["loaded"] = True
                _STATE["path"] = LIB_PATH
                _STATE["error"] = None
            except Exception as e:  # pragma: no cover - depends on the box
                _STATE["error"] = f"failed to load {LIB_PATH}: {e!r}"
        if not _STATE["loaded"] and raise_on_error:
            raise NativeExtensionError(_STATE["error"])
        return _STATE["loaded"]


def available() -> bool:
    return load(False)


def error() -> str | None:
    return _STATE["error"]


def reference_allowed() -> bool:
    return os.environ.get("DDIM_COLD_ALLOW_REFERENCE", "0") == "1"


_FORCE_REF = threading.local()


class force_reference:
    """Context manager: route GPU tensors to the PyTorch reference ops (tests / oracles)."""

    def __enter__(self):
        self.prev = getattr(_FORCE_REF, "on", False)
        _FORCE_REF.on = True
        return self

    def __exit__(self, *exc):
        _FORCE_REF.on = self.prev
        return False


def require_for(t: torch.Tensor) -> bool:
    """True -> use the HIP op for tensor ``t``; False -> use the reference op.

    Raises if ``t`` is on the GPU and the extension cannot be loaded (unless
    the reference path was explicitly allowed).
    """
    if not t.is_cuda or getattr(_FORCE_REF, "on", False):
        return False
    if load(False):
        return True
    if reference_allowed():
        return False
    raise NativeExtensionError(
        f"{_STATE['error']}; refusing to run GPU op on the PyTorch fallback "
        "(set DDIM_COLD_ALLOW_REFERENCE=1 to allow)")
