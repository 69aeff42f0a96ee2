"""Native build of the gfx950 extension (``pytorchvideo_accelerate_amd._C``).

No hipify, no ``torch.utils.cpp_extension.CUDAExtension`` (which would run hipify on ROCm): every
``csrc/kernels/*.hip`` file is compiled directly by ``hipcc --offload-arch=gfx950`` — twice, once per 16-bit
compute type (``-DPVA_F16=0``: bf16 operands, namespace ``pva_bf16``; ``-DPVA_F16=1``: fp16 operands, namespace
``pva_f16``; ``csrc/kernels/common.h``) — and linked with the pybind11 binding unit against libtorch.  Objects are cached by a hash of (source, headers, flags) so
re-builds only recompile what changed.  The resulting ``_C*.so`` lives in-tree next to this file (so it
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
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
CSRC = os.path.join(REPO, "csrc")
BUILD = os.path.join(REPO, "build", "obj")
ARCH = os.environ.get("PVA_OFFLOAD_ARCH", "gfx950")
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


def _headers_digest() -> str:
    h = hashlib.sha1()
    for f in sorted(glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)):
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def _compile(src: str, flags: list, hdr: str, force: bool, tag: str = "") -> str:
    with open(src, "rb") as fh:
        content = fh.read()
    key = hashlib.sha1(content + hdr.encode() + " ".join(flags).encode()).hexdigest()[:16]
    obj = os.path.join(BUILD, os.path.basename(src) + tag + "." + key + ".o")
    if os.path.exists(obj) and not force:
        return obj
    cmd = [HIPCC] + flags + ["-c", src, "-o", obj + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(obj + ".tmp", obj)
    return obj


def build(jobs: int = 0, force: bool = False, verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    _, tinc, tlib, abi = _torch_paths()
    pyinc = sysconfig.get_paths()["include"]
    common = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
              "-Wno-unused-result", "-Wno-unused-variable"]
    kern_flags = common + ["-ffp-contract=fast"]
    bind_flags = common + ["-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H", "-DUSE_ROCM=1",
                           "-D__HIP_PLATFORM_AMD__=1", f"-I{pyinc}"] + [f"-I{p}" for p in tinc]
    hdr = _headers_digest()
    kernels = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    runtime = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    jobs = jobs or min(16, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_compile, s, kern_flags + [f"-DPVA_F16={h}"], hdr, force, (".f16" if h else ".bf16"))
                for s in kernels for h in (0, 1)]
        futs += [ex.submit(_compile, s, bind_flags, hdr, force) for s in runtime]
        objs = [f.result() for f in futs]
    out = ext_path()
    libs = ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
            f"-L{ROCM_LIB}", f"-Wl,-rpath,{ROCM_LIB}", "-lrocprofiler-sdk-roctx"]   # ROCTx ranges
    stamp = hashlib.sha1(" ".join(objs).encode()).hexdigest()
    stamp_file = out + ".stamp"
    if os.path.exists(out) and not force and os.path.exists(stamp_file) and open(stamp_file).read() == stamp:
        return out
    cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}"] + objs + [f"-L{tlib}", f"-Wl,-rpath,{tlib}"] + libs + [
        "-o", out + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(out + ".tmp", out)
    with open(stamp_file, "w") as fh:
        fh.write(stamp)
    if verbose:
        print("built", out)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=0)
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args(argv)
    print(build(a.jobs, a.force, verbose=True))


if __name__ == "__main__":
    sys.exit(main())
