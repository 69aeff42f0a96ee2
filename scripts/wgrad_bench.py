"""Weight-gradient kernel micro-benchmark at the B=160 SlowFast-R50 gathered (non-1x1 / strided) shapes:
generic split-K kernel (conv_wgrad.hip) vs the row-table kernel (wgrad_rt_impl.h), best over tiles x split-K
targets x stage depth for each.

    python scripts/wgrad_bench.py [--batch 160] [--only name,...]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchvideo_accelerate_amd.ops._ext import require  # noqa: E402
from pytorchvideo_accelerate_amd.ops.conv import RT, ConvSpec, wgrad_splits  # noqa: E402

# name, cin, cout, k, stride, pad, (T, H, W) of the input, affine (input is a BN-ReLU recompute)
SHAPES = [
    ("s.res5.conv_a", 2048, 512, (3, 1, 1), (1, 1, 1), (1, 0, 0), (8, 7, 7), False),
    ("s.res5.conv_a0", 1280, 512, (3, 1, 1), (1, 1, 1), (1, 0, 0), (8, 14, 14), False),
    ("s.res4.conv_a", 1024, 256, (3, 1, 1), (1, 1, 1), (1, 0, 0), (8, 14, 14), False),
    ("s.res4.conv_a0", 640, 256, (3, 1, 1), (1, 1, 1), (1, 0, 0), (8, 28, 28), False),
    ("s.res5.conv_b", 512, 512, (1, 3, 3), (1, 1, 1), (0, 1, 1), (8, 7, 7), True),
    ("s.res4.conv_b", 256, 256, (1, 3, 3), (1, 1, 1), (0, 1, 1), (8, 14, 14), True),
    ("s.res5.b1_s2", 1280, 2048, (1, 1, 1), (1, 2, 2), (0, 0, 0), (8, 14, 14), False),
    ("s.res4.b1_s2", 640, 1024, (1, 1, 1), (1, 2, 2), (0, 0, 0), (8, 28, 28), False),
    ("s.res3.b1_s2", 320, 512, (1, 1, 1), (1, 2, 2), (0, 0, 0), (8, 56, 56), False),
    ("s.res4.conv_b_s2", 256, 256, (1, 3, 3), (1, 2, 2), (0, 1, 1), (8, 28, 28), True),
    ("f.res4.conv_a", 128, 32, (3, 1, 1), (1, 1, 1), (1, 0, 0), (32, 14, 14), False),
    ("f.res3.conv_a", 64, 16, (3, 1, 1), (1, 1, 1), (1, 0, 0), (32, 28, 28), False),
]


def timeit(fn, iters=5):
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
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    C = require()
    dev = torch.device("cuda")
    only = set(a.only.split(",")) if a.only else None
    for name, cin, cout, k, st, pd, (T, H, W), aff in SHAPES:
        if only and name not in only:
            continue
        spec = ConvSpec(cin, cout, k, st, pd)
        To, Ho, Wo = spec.out_dims(T, H, W)
        P = a.batch * To * Ho * Wo
        Mi = a.batch * T * H * W
        x = torch.randn(Mi, cin, device=dev).to(torch.bfloat16)
        dy = torch.randn(P, cout, device=dev).to(torch.bfloat16)
        sc = torch.rand(cin, device=dev) + 0.5 if aff else None
        sh = torch.randn(cin, device=dev) * 0.1 if aff else None
        K = spec.taps * cin
        acc = torch.zeros(cout * K, device=dev)
        flops = 2.0 * P * cout * K
        res = {}
        for rt in (False, True):
            best = None
            for t in range(2, 8):
                vw = (t & 3) | (8 if t >= 4 else 0)
                for tbi, tb in enumerate((512, 1024, 2048, 4096)):
                    for bp in (0, 4):
                        splits, pps = wgrad_splits(P, cout, K, target_blocks=tb, variant=vw)
                        g = [P, cout, K, cin, cout, cin, T, H, W, To, Ho, Wo, *k, *st, *pd, splits, pps]
                        word = vw | bp | (RT if rt else 0)
                        us = timeit(lambda: C.conv_wgrad(dy, x, acc, sc, sh, 2 if aff else 0, g, 8, 0, word, 0, None))
                        if best is None or us < best[0]:
                            best = (us, t, tb, bp)
            res[rt] = best
        o, n = res[False], res[True]
        print("%-18s P=%8d Cout=%5d K=%5d  generic %8.1f us %6.0f TF/s (tile %d tb %d bp %d) | row-table %8.1f us "
              "%6.0f TF/s (tile %d tb %d bp %d)  x%.2f" % (name, P, cout, K, o[0], flops / o[0] / 1e6, o[1], o[2], o[3],
                                                          n[0], flops / n[0] / 1e6, n[1], n[2], n[3], o[0] / n[0]),
              flush=True)


if __name__ == "__main__":
    main()
