"""Fast-stem (k(5,7,7), Cout 8) s2d kernels at the B=160 SlowFast-R50 shape: forward and weight gradient, per kernel
variant (stem_pair is read per launch).  Round 4 also timed a two-pair weight-gradient kernel here (8 waves,
12-frame ring, each LDS fragment feeding both pairs): 2412 vs 1956 us for the pair kernel — removed.
    python scripts/stem_bench.py [--batch 160] [--iters 10]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchvideo_accelerate_amd.ops._ext import require  # noqa


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=160)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    C = require()
    dev = torch.device("cuda")
    N, T, Hs, kt, cout = a.batch, 32, 112, 5, 8
    M = N * T * Hs * Hs
    xs = (torch.randn(M, 16, device=dev) * 0.5).to(torch.bfloat16)
    dy = torch.randn(M, cout, device=dev).to(torch.bfloat16)
    wp = torch.zeros(16 * kt * 256, device=dev, dtype=torch.bfloat16)
    C.stem_pack((torch.randn(cout, 3, kt, 7, 7, device=dev) * 0.05).contiguous(), wp, cout, kt)
    y = torch.empty(M, cout, device=dev, dtype=torch.bfloat16)
    stats = torch.empty(C.stem_tiles(Hs, Hs, N), 2, cout, device=dev)
    acc = torch.zeros(cout * kt * 256, device=dev)
    flop = 2.0 * M * cout * 3 * kt * 49
    ref = None
    for pair in ("0", "1", "0", "1"):   # twice each: the first launches of a process run at lower clocks
        os.environ["PVA_ARMS"] = f"stem_pair={pair}"
        tf = timeit(lambda: C.stem_fwd(xs, wp, y, stats, [N, T, Hs, Hs], cout, kt), a.iters)
        acc.zero_()
        tw = timeit(lambda: C.stem_wgrad(xs, dy, acc, [N, T, Hs, Hs], cout, kt), a.iters)
        acc.zero_()
        C.stem_wgrad(xs, dy, acc, [N, T, Hs, Hs], cout, kt)
        torch.cuda.synchronize()
        if ref is None:
            ref = acc.clone()
        err = ((acc - ref).norm() / ref.norm()).item()
        print(f"pair={pair}: fwd {tf:8.1f} us ({flop / tf / 1e6:6.1f} TF/s)  wgrad {tw:8.1f} us "
              f"({flop / tw / 1e6:6.1f} TF/s)  wgrad rel-diff vs one-frame kernel {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
