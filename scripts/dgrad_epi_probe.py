"""Epilogue cost of the wide-output dgrads (res4 / res5 conv_a: dX has 4x the channels of dY, K = 3 x Cout):
time every autotuner candidate of the dgrad with a plain store (accum=0) and with the accumulate epilogue
(accum=1: read + add + store of dX), next to the forward conv of the same layer (same FLOPs, narrow output).

    python scripts/dgrad_epi_probe.py [--batch 160]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchvideo_accelerate_amd.ops.conv import Act, ConvSpec, dgrad_phases, fwd_geometry, pack_weight  # noqa
from pytorchvideo_accelerate_amd.ops.tune import ConvTuner, describe  # noqa

SHAPES = [
    ("s.res4.conv_a", 1024, 256, (3, 1, 1), (1, 0, 0), (8, 14, 14)),
    ("s.res4.conv_a0", 640, 256, (3, 1, 1), (1, 0, 0), (8, 28, 28)),
    ("s.res5.conv_a", 2048, 512, (3, 1, 1), (1, 0, 0), (8, 7, 7)),
]


def timeit(fn, iters=10):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=160)
    a = ap.parse_args()
    from pytorchvideo_accelerate_amd.ops._ext import require
    C = require()
    tuner = ConvTuner(C)
    dev = "cuda"
    for name, cin, cout, k, pd, (T, H, W) in SHAPES:
        spec = ConvSpec(cin, cout, k, (1, 1, 1), pd)
        N = a.batch
        M = N * T * H * W
        w = torch.randn(cout, cin, *k, device=dev) * 0.05
        wf, wd = pack_weight(w, spec)
        x = torch.randn(M, cin, device=dev).to(torch.bfloat16)
        y = torch.empty(M, cout, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(M, cout, device=dev).to(torch.bfloat16)
        dx = torch.randn(M, cin, device=dev).to(torch.bfloat16)
        flops = spec.flops(N, T, H, W)
        gf = fwd_geometry(spec, N, T, H, W, cin, cout)
        (gd,) = list(dgrad_phases(spec, N, (T, H, W), (T, H, W), cout, cin))
        rows = []
        for label, g, src, wt, dst, acc in (("fwd", gf, x, wf, y, 0), ("dgrad store", gd, dy, wd, dx, 0),
                                           ("dgrad accum", gd, dy, wd, dx, 1)):
            best = None
            for cfg in tuner.candidates(g, 8, 0, False, True, True, acc == 0):
                t = timeit(lambda: C.conv_igemm(src, wt, dst, None, None, None, 0, acc, g, 8, cfg))
                if best is None or t < best[0]:
                    best = (t, cfg)
            rows.append((label, best))
        out_mb = M * cin * 2 / 1e6
        print(f"{name} B={N} M={M} Cin={cin} Cout={cout} (dX {out_mb:.0f} MB bf16, {flops / 1e12:.3f} TFLOP)")
        for label, (t, cfg) in rows:
            print(f"  {label:12s} {t:8.1f} us {flops / t / 1e6:7.1f} TF/s  [{describe(cfg)}]")


if __name__ == "__main__":
    main()
