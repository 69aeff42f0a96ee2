"""Per-conv-class microbenchmark of the gfx950 conv kernels (fwd / dgrad / wgrad TFLOP/s).

    python scripts/conv_bench.py [--batch 8] [--iters 20]
Shapes are the SlowFast-R50 32x2x224 classes of SURVEY.md Appendix B.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchvideo_accelerate_amd.ops.conv import Act, ConvSpec, conv_dgrad, conv_fwd, conv_wgrad, pack_weight  # noqa

# name, cin, cout, k, stride, pad, (T, H, W)
SHAPES = [
    ("s.res2.conv_b", 64, 64, (1, 3, 3), (1, 1, 1), (0, 1, 1), (8, 56, 56)),
    ("s.res2.conv_c", 64, 256, (1, 1, 1), (1, 1, 1), (0, 0, 0), (8, 56, 56)),
    ("s.res3.conv_b", 128, 128, (1, 3, 3), (1, 1, 1), (0, 1, 1), (8, 28, 28)),
    ("s.res4.conv_a0", 640, 256, (3, 1, 1), (1, 1, 1), (1, 0, 0), (8, 28, 28)),
    ("s.res4.conv_a", 1024, 256, (3, 1, 1), (1, 1, 1), (1, 0, 0), (8, 14, 14)),
    ("s.res4.conv_b", 256, 256, (1, 3, 3), (1, 1, 1), (0, 1, 1), (8, 14, 14)),
    ("s.res4.conv_c", 256, 1024, (1, 1, 1), (1, 1, 1), (0, 0, 0), (8, 14, 14)),
    ("s.res5.conv_a", 2048, 512, (3, 1, 1), (1, 1, 1), (1, 0, 0), (8, 7, 7)),
    ("s.res5.conv_b", 512, 512, (1, 3, 3), (1, 1, 1), (0, 1, 1), (8, 7, 7)),
    ("s.res3.b1_s2", 320, 512, (1, 1, 1), (1, 2, 2), (0, 0, 0), (8, 56, 56)),
    ("s.res3.conv_b_s2", 128, 128, (1, 3, 3), (1, 2, 2), (0, 1, 1), (8, 56, 56)),
    ("f.res2.conv_b", 8, 8, (1, 3, 3), (1, 1, 1), (0, 1, 1), (32, 56, 56)),
    ("f.res2.conv_a", 32, 8, (3, 1, 1), (1, 1, 1), (1, 0, 0), (32, 56, 56)),
    ("f.res3.conv_c", 16, 64, (1, 1, 1), (1, 1, 1), (0, 0, 0), (32, 28, 28)),
    ("f.res4.conv_b", 32, 32, (1, 3, 3), (1, 1, 1), (0, 1, 1), (32, 14, 14)),
    ("fuse1", 32, 64, (7, 1, 1), (4, 1, 1), (3, 0, 0), (32, 56, 56)),
    ("s.stem", 3, 64, (1, 7, 7), (1, 2, 2), (0, 3, 3), (8, 224, 224)),
    ("f.stem", 3, 8, (5, 7, 7), (1, 2, 2), (2, 3, 3), (32, 224, 224)),
]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--bk", type=int, default=-1)
    ap.add_argument("--affine", type=int, default=0, help="1: forward applies consumer-side BN+ReLU to its input")
    ap.add_argument("--ut", type=int, default=1, help="uniform-tap loader: 0 never, 1 heuristic (default), 2 always")
    a = ap.parse_args()
    from pytorchvideo_accelerate_amd.ops._ext import require
    if a.bk > 0:
        require().conv_set_bk(a.bk)
    require().conv_set_ut(a.ut)
    dev = "cuda"
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    print(f"{'layer':18s} {'M':>8s} {'N':>5s} {'K':>5s} | {'fwd us':>8s} {'TF':>6s} | {'dgrad us':>8s} {'TF':>6s} | {'wgrad us':>8s} {'TF':>6s}")
    for name, cin, cout, k, st, pd, (T, H, W) in SHAPES:
        if a.only and a.only not in name:
            continue
        spec = ConvSpec(cin, cout, k, st, pd, cin_pad=4 if cin == 3 else 0)
        N = a.batch
        x = torch.randn(N, cin, T, H, W, device=dev)
        w = torch.randn(cout, cin, *k, device=dev) * 0.05
        xa = Act.from_ncthw(x, spec.cin_pad)
        wf, wd = pack_weight(w, spec)
        To, Ho, Wo = spec.out_dims(T, H, W)
        M = N * To * Ho * Wo
        flops = spec.flops(N, T, H, W)
        out = torch.empty(M, cout, device=dev, dtype=torch.bfloat16)
        if a.affine:
            sc = torch.rand(spec.cin_pad or cin, device=dev) + 0.5
            sh = torch.randn(spec.cin_pad or cin, device=dev) * 0.1
            tf = timeit(lambda: conv_fwd(xa, wf, spec, out=out, in_scale=sc, in_shift=sh, in_relu=True), a.iters)
        else:
            tf = timeit(lambda: conv_fwd(xa, wf, spec, out=out), a.iters)
        dy = Act(torch.randn(M, cout, device=dev).to(torch.bfloat16), N, To, Ho, Wo)
        if cin % 8 == 0:
            dx = torch.empty(xa.M, cin, device=dev, dtype=torch.bfloat16)
            td = timeit(lambda: conv_dgrad(dy, wd, spec, (T, H, W), out=dx), a.iters)
        else:
            td = float("nan")
        g = torch.zeros_like(w)
        ws = torch.zeros(cout * spec.taps * spec.cin_pad, device=dev)
        tw = timeit(lambda: conv_wgrad(dy, xa, spec, g, workspace=ws), a.iters)
        tot["fwd"] += tf
        tot["dgrad"] += 0 if td != td else td
        tot["wgrad"] += tw
        K = spec.taps * spec.cin_pad
        print(f"{name:18s} {M:8d} {cout:5d} {K:5d} | {tf*1e3:8.1f} {flops/tf/1e9:6.1f} | {td*1e3:8.1f} {flops/td/1e9:6.1f} | {tw*1e3:8.1f} {flops/tw/1e9:6.1f}")
    print("totals ms", {k: round(v, 3) for k, v in tot.items()})


if __name__ == "__main__":
    main()
