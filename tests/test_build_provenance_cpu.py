"""Binary provenance: the extension embeds the build id of the source tree it was linked
from; ``build()`` relinks whenever that id differs and the loader refuses a stale binary."""
import os
import shutil

import pytest

from pytorchvideo_accelerate_amd import _build
from pytorchvideo_accelerate_amd.ops import _ext

HAVE_SO = os.path.exists(_build.ext_path())
HAVE_HIPCC = os.path.exists(_build.HIPCC)


def _copy_tree(tmp_path):
    csrc = tmp_path / "csrc"
    shutil.copytree(_build.CSRC, csrc)
    return str(csrc)


def _touch_kernel(csrc):
    with open(os.path.join(csrc, "kernels", "optim_pack.hip"), "a") as f:
        f.write("\n// provenance test edit\n")


def test_tree_id_tracks_sources(tmp_path):
    csrc = _copy_tree(tmp_path)
    a = _build.tree_id(csrc)
    assert a == _build.tree_id(_build.CSRC)
    _touch_kernel(csrc)
    assert _build.tree_id(csrc) != a
    # headers count too
    csrc2 = _copy_tree(tmp_path / "b")
    with open(os.path.join(csrc2, "kernels", "common.h"), "a") as f:
        f.write("\n")
    assert _build.tree_id(csrc2) != a


@pytest.mark.skipif(not HAVE_SO, reason="extension not built")
def test_shipped_binary_matches_tree():
    ok, emb, want = _build.check()
    assert ok, f"shipped .so built from {emb}, tree is {want}"


@pytest.mark.skipif(not HAVE_SO, reason="extension not built")
def test_stale_binary_is_refused(tmp_path, monkeypatch):
    csrc = _copy_tree(tmp_path)
    _touch_kernel(csrc)
    monkeypatch.setattr(_build, "CSRC", csrc)
    ok, emb, want = _build.check()
    assert not ok and emb != want
    monkeypatch.setenv("PVA_AUTOBUILD", "0")
    with pytest.raises(_ext.StaleExtensionError):
        _ext.verify()
    monkeypatch.setattr(_ext, "_C", None)
    with pytest.raises(_ext.StaleExtensionError):
        _ext.load()


@pytest.mark.skipif(not (HAVE_SO and HAVE_HIPCC and os.path.isdir(_build.BUILD)), reason="needs hipcc and a built extension (object cache)")
def test_build_relinks_after_kernel_edit(tmp_path):
    csrc = _copy_tree(tmp_path)
    bdir = tmp_path / "obj"
    bdir.mkdir()
    for f in os.listdir(_build.BUILD):          # reuse the object cache: only the edited kernel recompiles
        if f.endswith(".o"):
            os.link(os.path.join(_build.BUILD, f), bdir / f)
    out = str(tmp_path / "_C.so")
    shutil.copy(_build.ext_path(), out)
    # unchanged tree: nothing relinked
    m0 = os.stat(out).st_mtime_ns
    _build.build(csrc=csrc, build_dir=str(bdir), out=out)
    assert os.stat(out).st_mtime_ns == m0
    _touch_kernel(csrc)
    assert _build.embedded_id(out) != _build.tree_id(csrc)
    _build.build(csrc=csrc, build_dir=str(bdir), out=out)
    assert _build.embedded_id(out) == _build.tree_id(csrc)
    assert os.stat(out).st_mtime_ns != m0


def test_tree_id_covers_real_flags_and_torch_version(monkeypatch):
    """Advisor r5: the build id hashes the flag lists build() actually uses and the torch version, so a changed
    compile flag or a torch upgrade makes the shipped binary stale (no hand-written flags string)."""
    from pytorchvideo_accelerate_amd import _build
    import torch
    base = _build.tree_id()
    orig = _build._flags

    def more_flags():
        c, k, b = orig()
        return c, k + ["-mcumode"], b
    monkeypatch.setattr(_build, "_flags", more_flags)
    assert _build.tree_id() != base
    monkeypatch.setattr(_build, "_flags", orig)
    monkeypatch.setattr(torch, "__version__", torch.__version__ + "+other")
    assert _build.tree_id() != base
    monkeypatch.undo()
    assert _build.tree_id() == base


def test_embedded_id_is_cached_and_mmap_scanned(tmp_path):
    from pytorchvideo_accelerate_amd import _build
    p = tmp_path / "x.so"
    p.write_bytes(b"\0" * 1000 + _build.ID_MARK + b"a" * 40 + b"\0" * 10)
    assert _build.embedded_id(str(p)) == "a" * 40
    assert any(k[0] == str(p) for k in _build._EMB_CACHE)
    p.write_bytes(b"\0" * 5000)   # new size -> new cache key -> rescanned
    assert _build.embedded_id(str(p)) is None
