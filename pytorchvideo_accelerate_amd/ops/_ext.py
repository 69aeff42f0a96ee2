"""Loader for the in-tree gfx950 extension.

The HIP path must be the one that runs on a GPU box: if the extension cannot be imported while a GPU
is present we raise (no silent eager fallback).  On a CPU-only host ``available()`` is False and the
framework uses its pure-PyTorch reference path (``models/reference.py``).

Provenance: before importing, the binary's embedded build id (``_build.embedded_id``) is compared with the id of
the ``csrc/`` tree next to the package (``_build.tree_id``).  A stale binary is rebuilt when ``PVA_AUTOBUILD=1``
and refused (``StaleExtensionError``) otherwise — a kernel edit can never run against an old ``.so`` unnoticed.
"""
from __future__ import annotations

import os

_C = None
_ERR = None


class StaleExtensionError(RuntimeError):
    pass


def verify() -> None:
    """Raise StaleExtensionError when the built ``.so`` was not linked from this source tree."""
    from .. import _build
    path = _build.ext_path()
    if not os.path.exists(path):
        return
    ok, emb, want = _build.check(path)
    if not ok:
        raise StaleExtensionError(f"{path} was built from tree {emb}, the csrc/ tree is {want}: rebuild with "
                                  "`python -m pytorchvideo_accelerate_amd._build` (or set PVA_AUTOBUILD=1)")


def load(build_if_missing: bool = False):
    global _C, _ERR
    if _C is not None:
        return _C
    try:
        verify()
    except StaleExtensionError:
        if os.environ.get("PVA_AUTOBUILD", "0") != "1":
            raise
        from .._build import build
        build()
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
