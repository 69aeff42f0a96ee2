"""Forward conv microbenchmark with an explicit launch configuration word (for A/B and PMC runs).

    python scripts/direct_bench.py --shape f.res2.conv_b --batch 96 --cfg direct2048 [--affine 1]
``--cfg``: direct512 | direct2048 | heuristic | <int config word> (ops/tune.py)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchvideo_accelerate_amd.ops.conv import Act, ConvSpec, fwd_geometry, pack_weight  # noqa: E402
from pytorchvideo_accelerate_amd.ops import tune  # noqa: E402

SHAPES = {
    "f.res2.conv_b": (8, 8, (1, 3, 3), (1, 1, 1), (0, 1, 1), (32, 56, 56)),
    "f.res2.conv_a": (32, 8, (3, 1, 1), (1, 1, 1), (1, 0, 0), (32, 56, 56)),
    "f.res2.conv_c": (8, 32, (1, 1, 1), (1, 1, 1), (0, 0, 0), (32, 56, 56)),
    "f.res3.conv_b": (16, 16, (1, 3, 3), (1, 1, 1), (0, 1, 1), (32, 28, 28)),
    "s.res2.conv_a0": (80, 64, (1, 1, 1), (1, 1, 1), (0, 0, 0), (8, 56, 56)),
    "s.res2.conv_c": (64, 256, (1, 1, 1), (1, 1, 1), (0, 0, 0), (8, 56, 56)),
    "s.res3.conv_c": (128, 512, (1, 1, 1), (1, 1, 1), (0, 0, 0), (8, 28, 28)),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="f.res2.conv_b")
    ap.add_argument("--batch", type=int, default=96)
    ap.add_argument("--cfg", default="direct2048")
    ap.add_argument("--affine", type=int, default=1)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--nostats", action="store_true")
    ap.add_argument("--nostore", action="store_true", help="debug builds only: accum=2 skips the output store")
    a = ap.parse_args()
    from pytorchvideo_accelerate_amd.ops._ext import require
    C = require()
    cin, cout, k, st, pd, (T, H, W) = SHAPES[a.shape]
    spec = ConvSpec(cin, cout, k, st, pd)
    dev = "cuda"
    N = a.batch
    x = torch.randn(N * T * H * W, cin, device=dev).to(torch.bfloat16)
    xa = Act(x, N, T, H, W)
    wf, _ = pack_weight(torch.randn(cout, cin, *k, device=dev) * 0.05, spec)
    To, Ho, Wo = spec.out_dims(T, H, W)
    M = N * To * Ho * Wo
    y = torch.empty(M, cout, device=dev, dtype=torch.bfloat16)
    stats = torch.empty((M + 127) // 128, 2, cout, device=dev)
    sc = torch.rand(cin, device=dev) + 0.5
    sh = torch.randn(cin, device=dev) * 0.1
    g = fwd_geometry(spec, N, T, H, W, cin, cout)
    cfg = {"direct512": tune.EXPLICIT | tune.DIRECT, "direct2048": tune.EXPLICIT | tune.DIRECT | tune.DIRECT_2K,
           "heuristic": -1}.get(a.cfg)
    cfg = int(a.cfg) if cfg is None else cfg

    def run():
        C.conv_igemm(xa.t, wf, y, None if a.nostats else stats, sc if a.affine else None, sh if a.affine else None, 2 if a.affine else 0,
                     2 if a.nostore else 0, g, 8, cfg)
    for _ in range(3):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        run()
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / a.iters
    gb = (M * cin + M * cout) * 2 / 1e9
    print(f"{a.shape} B={N} cfg={tune.describe(cfg)}: {us:.1f} us, {gb / us * 1e3:.2f} TB/s (min traffic {gb:.3f} GB)")


if __name__ == "__main__":
    main()
