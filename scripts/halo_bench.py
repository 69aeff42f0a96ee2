"""Times the (1,3,3) conv_b kernels at the B=160 SlowFast-R50 shapes: the halo-staged conv (csrc/kernels/conv_halo.hip,
both n-tiles) against the best implicit-GEMM / direct configuration the autotuner knows, forward (BN+ReLU prologue
+ statistics) and dgrad, plus the box-staged weight gradient.  Prints microseconds and TF/s per configuration.

    python scripts/halo_bench.py [--batch 160] [--only 64,128]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchvideo_accelerate_amd.ops.conv import (BOX, Act, ConvSpec, conv_dgrad, conv_fwd, conv_wgrad,  # noqa: E402
                                                  dgrad_phases, fwd_geometry, pack_weight)
from pytorchvideo_accelerate_amd.ops.tune import ConvTuner, describe  # noqa: E402

# channels, T, H(=W)  (slow res2..res4, fast res2..res4)
SHAPES = [(64, 8, 56), (128, 8, 28), (256, 8, 14), (8, 32, 56), (16, 32, 28), (32, 32, 14)]


def timeit(fn, iters=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=160)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    from pytorchvideo_accelerate_amd.ops._ext import require
    Cm = require()
    tuner = ConvTuner(Cm)
    dev = torch.device("cuda")
    only = {int(v) for v in a.only.split(",") if v}
    for C, T, H in SHAPES:
        if only and C not in only:
            continue
        N = a.batch
        spec = ConvSpec(C, C, (1, 3, 3), (1, 1, 1), (0, 1, 1))
        M = N * T * H * H
        x = torch.randn(M, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(C, C, 1, 3, 3, device=dev) / (9 * C) ** 0.5)
        wf, wd = pack_weight(w, spec)
        xa = Act(x, N, T, H, H)
        sc = torch.rand(C, device=dev) + 0.5
        sh = torch.randn(C, device=dev) * 0.3
        flop = 2.0 * M * C * C * 9
        g = fwd_geometry(spec, N, T, H, H, C, C)
        stats = torch.empty((M + 127) // 128, 2, C, device=dev)
        out = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
        res = []
        for cfg in tuner.candidates(g, 8, aff=2):
            t = timeit(lambda: conv_fwd(xa, wf, spec, out=out, stats=stats, in_scale=sc, in_shift=sh, cfg=cfg))
            res.append((t, describe(cfg)))
        res.sort()
        print(f"C={C:3d} {T}x{H}x{H} fwd  : " + "  ".join(f"{d}={t:.0f}us({flop / t / 1e6:.0f}TF)" for t, d in res[:4]),
              flush=True)
        gd = dgrad_phases(spec, N, (T, H, H), (T, H, H), C, C)[0]
        res = []
        for cfg in tuner.candidates(gd, 8):
            t = timeit(lambda: conv_dgrad(xa, wd, spec, (T, H, H), out=out, cfg=cfg))
            res.append((t, describe(cfg)))
        res.sort()
        print(f"C={C:3d} {T}x{H}x{H} dgrad: " + "  ".join(f"{d}={t:.0f}us({flop / t / 1e6:.0f}TF)" for t, d in res[:4]),
              flush=True)
        grad = torch.empty(C, C, 1, 3, 3, device=dev)
        t = timeit(lambda: conv_wgrad(xa, xa, spec, grad, in_scale=sc, in_shift=sh, variant=BOX))
        print(f"C={C:3d} {T}x{H}x{H} wgrad: box={t:.0f}us({flop / t / 1e6:.0f}TF)", flush=True)


if __name__ == "__main__":
    main()
