"""Native build of the gfx950 extension (``pytorchvideo_accelerate_amd._C``).

No hipify, no ``torch.utils.cpp_extension.CUDAExtension`` (which would run hipify on ROCm): every
``csrc/kernels/*.hip`` file is compiled directly by ``hipcc --offload-arch=gfx950`` — twice, once per 16-bit
compute type (``-DPVA_F16=0``: bf16 operands, namespace ``pva_bf16``; ``-DPVA_F16=1``: fp16 operands, namespace
``pva_f16``; ``csrc/kernels/common.h``) — and linked with the pybind11 binding unit against libtorch.  Objects are cached by a hash of (source, headers, flags) so
re-builds only recompile what changed.  The binary carries the build id of the tree it was linked from
(``tree_id``: sources, headers, flags; ``_C.build_id()``); ``build()`` relinks whenever it differs and the loader
(``ops/_ext.py``) refuses a stale binary.  The resulting ``_C*.so`` lives in-tree next to this file (so it
travels to the GPU box with the repository snapshot).

    python -m pytorchvideo_accelerate_amd._build [--jobs N] [--force]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import subprocess
import sys
import re
import sysconfig
from typing import Optional, Tuple

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
CSRC = os.path.join(REPO, "csrc")
BUILD = os.path.join(REPO, "build", "obj")
ARCH = "gfx950"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ROCM_LIB = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib")


def ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG_DIR, "_C" + suffix)


def _torch_paths():
    import torch

    root = os.path.dirname(torch.__file__)
    inc = [os.path.join(root, "include"), os.path.join(root, "include", "torch", "csrc", "api", "include")]
    return root, inc, os.path.join(root, "lib"), int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _headers_digest(csrc: str = CSRC) -> str:
    h = hashlib.sha1()
    for f in sorted(glob.glob(os.path.join(csrc, "**", "*.h"), recursive=True)):
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


ID_MARK = b"PVA_BUILD_ID:"
_ID_RE = re.compile(re.escape(ID_MARK) + rb"([0-9a-f]{40})")


def _flags():
    """(common, kernel, binding) compile flags — the one source of truth for ``build()`` and ``tree_id()``."""
    _, tinc, _, abi = _torch_paths()
    pyinc = sysconfig.get_paths()["include"]
    common = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
              "-Wno-unused-result", "-Wno-unused-variable"]
    kern = common + ["-ffp-contract=fast"]
    bind = common + ["-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H", "-DUSE_ROCM=1",
                     "-D__HIP_PLATFORM_AMD__=1", f"-I{pyinc}"] + [f"-I{p}" for p in tinc]
    return common, kern, bind


def flags_signature() -> str:
    """Everything that changes the generated code: the real flag lists (include paths dropped — they only say where
    the same headers live), the per-type builds, the torch version (its headers are compiled into the bindings)."""
    import torch
    common, kern, bind = _flags()
    keep = lambda fl: [f for f in fl if not f.startswith("-I")]   # noqa: E731
    return "|".join([" ".join(keep(common)), " ".join(keep(kern)), " ".join(keep(bind)), "PVA_F16=0,1;fp32:0",
                     "torch=" + torch.__version__])


def tree_id(csrc: str = CSRC) -> str:
    """Build id of a source tree: sha1 over every csrc source/header (relative path + bytes) and the flags.
    Compiled into the extension (``_C.build_id()``), so a binary can be checked against the tree it ships with."""
    h = hashlib.sha1(flags_signature().encode())
    files = []
    for ext in ("*.hip", "*.h", "*.cpp"):
        files += glob.glob(os.path.join(csrc, "**", ext), recursive=True)
    for f in sorted(files, key=lambda f: os.path.relpath(f, csrc)):
        h.update(os.path.relpath(f, csrc).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()


_EMB_CACHE = {}


def embedded_id(so_path: str) -> Optional[str]:
    """The build id compiled into a built ``_C*.so`` (read from the file, without importing it), or None.
    The file is scanned through ``mmap`` (no 40 MB read) and the answer cached per (path, size, mtime)."""
    import mmap
    try:
        st = os.stat(so_path)
    except OSError:
        return None
    key = (os.path.abspath(so_path), st.st_size, st.st_mtime_ns)
    if key in _EMB_CACHE:
        return _EMB_CACHE[key]
    try:
        with open(so_path, "rb") as fh, mmap.mmap(fh.fileno(), 0, access=mmap.ACCESS_READ) as mm:
            m = _ID_RE.search(mm)
            val = m.group(1).decode() if m else None
    except (OSError, ValueError):
        return None
    _EMB_CACHE[key] = val
    return val


def check(so_path: Optional[str] = None, csrc: Optional[str] = None) -> Tuple[bool, Optional[str], Optional[str]]:
    """(up to date, embedded id, tree id).  Without a source tree next to the package nothing can be compared:
    that counts as up to date (an installed copy)."""
    so_path = so_path or ext_path()
    csrc = csrc or CSRC
    emb = embedded_id(so_path)
    if not os.path.isdir(csrc):
        return emb is not None, emb, None
    want = tree_id(csrc)
    return emb == want, emb, want


def _compile(src: str, flags: list, hdr: str, force: bool, tag: str = "", build_dir: str = BUILD) -> str:
    with open(src, "rb") as fh:
        content = fh.read()
    key = hashlib.sha1(content + hdr.encode() + " ".join(flags).encode()).hexdigest()[:16]
    obj = os.path.join(build_dir, os.path.basename(src) + tag + "." + key + ".o")
    if os.path.exists(obj) and not force:
        return obj
    tmp = f"{obj}.{os.getpid()}.tmp"
    cmd = [HIPCC] + flags + ["-c", src, "-o", tmp]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, obj)
    return obj


def build(jobs: int = 0, force: bool = False, verbose: bool = False, csrc: str = CSRC, build_dir: str = BUILD,
          out: Optional[str] = None) -> str:
    """Compile (object cache keyed by content) and relink whenever the binary's embedded build id differs from
    the tree's — never trusts a side file.  ``csrc`` / ``build_dir`` / ``out`` let a test build a copy of the tree.
    Serialised across processes by a lock file in ``build_dir`` (every torchrun rank may find a stale binary at
    once under ``PVA_AUTOBUILD=1``): the first builds, the others then see an up-to-date binary and return."""
    import fcntl
    os.makedirs(build_dir, exist_ok=True)
    with open(os.path.join(build_dir, ".build.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            return _build_locked(jobs, force, verbose, csrc, build_dir, out)
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)


def _build_locked(jobs, force, verbose, csrc, build_dir, out) -> str:
    _, _, tlib, _ = _torch_paths()
    common, kern_flags, bind_flags = _flags()
    out = out or ext_path()
    bid = tree_id(csrc)
    if os.path.exists(out) and not force and embedded_id(out) == bid:
        return out
    hdr = _headers_digest(csrc)
    kernels = sorted(glob.glob(os.path.join(csrc, "kernels", "*.hip")))
    kernels32 = sorted(glob.glob(os.path.join(csrc, "fp32", "*.hip")))   # fp32 path: one build (split-bf16 MFMA)
    runtime = sorted(glob.glob(os.path.join(csrc, "runtime", "*.cpp")))
    id_src = os.path.join(build_dir, f"build_id.{bid}.cpp")
    if not os.path.exists(id_src):
        with open(f"{id_src}.{os.getpid()}.tmp", "w") as fh:
            fh.write('extern "C" const char pva_build_id_str[] = "%s%s";\n' % (ID_MARK.decode(), bid))
        os.replace(f"{id_src}.{os.getpid()}.tmp", id_src)
    jobs = jobs or min(16, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_compile, s, kern_flags + [f"-DPVA_F16={h}"], hdr, force, (".f16" if h else ".bf16"), build_dir)
                for s in kernels for h in (0, 1)]
        futs += [ex.submit(_compile, s, kern_flags + ["-DPVA_F16=0"], hdr, force, ".f32", build_dir) for s in kernels32]
        futs += [ex.submit(_compile, s, bind_flags, hdr, force, "", build_dir) for s in runtime]
        futs.append(ex.submit(_compile, id_src, common, "", force, "", build_dir))
        objs = [f.result() for f in futs]
    libs = ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
            f"-L{ROCM_LIB}", f"-Wl,-rpath,{ROCM_LIB}", "-lrocprofiler-sdk-roctx",   # ROCTx ranges
            "-ldl"]   # RCCL: bound at run time to torch's copy (csrc/runtime/rccl_comm.cpp)
    tmp = f"{out}.{os.getpid()}.tmp"
    cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}"] + objs + [f"-L{tlib}", f"-Wl,-rpath,{tlib}"] + libs + [
        "-o", tmp]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)
    if embedded_id(out) != bid:
        raise RuntimeError(f"linked {out} but its embedded build id is not {bid}")
    if verbose:
        print("built", out, "build id", bid)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=0)
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args(argv)
    print(build(a.jobs, a.force, verbose=True))


if __name__ == "__main__":
    sys.exit(main())
