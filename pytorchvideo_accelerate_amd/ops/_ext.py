"""Loader for the in-tree gfx950 extension.

The HIP path must be the one that runs on a GPU box: if the extension cannot be imported while a GPU
is present we raise (no silent eager fallback).  On a CPU-only host ``available()`` is False and the
framework uses its pure-PyTorch reference path (``models/reference.py``).
"""
from __future__ import annotations

import os

_C = None
_ERR = None


def load(build_if_missing: bool = False):
    global _C, _ERR
    if _C is not None:
        return _C
    try:
        from .. import _C as mod  # type: ignore
        _C = mod
        return _C
    except ImportError as e:  # pragma: no cover - exercised on fresh checkouts
        _ERR = e
        if build_if_missing:
            from .._build import build
            build()
            from .. import _C as mod  # type: ignore
            _C = mod
            return _C
        return None


def available() -> bool:
    return load() is not None


def require():
    """Return the extension or fail loudly (used by every GPU op)."""
    mod = load(build_if_missing=os.environ.get("PVA_AUTOBUILD", "1") == "1")
    if mod is None:
        raise RuntimeError(f"pytorchvideo_accelerate_amd._C (gfx950 kernels) is not built: {_ERR}. "
                           "Run `python -m pytorchvideo_accelerate_amd._build`.")
    return mod
