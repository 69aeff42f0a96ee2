"""Fast-stem weight gradient at the headline shape (SlowFast-R50 32x2x224, B=160: s2d input [160, 32, 112, 112, 16],
dY [.., 8]), the rolling-fragment frame-pair kernel (default) against the one-tap-row-per-wave form
(stem_roll=0) and the rolling form with intrinsic transpose reads (stem_async=0); both read per launch.
Prints the mean kernel time of each and the results' relative differences."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from pytorchvideo_accelerate_amd.ops._ext import require
    C = require()
    dev = torch.device("cuda")
    N, T, H, cout, kt = int(os.environ.get("B", 160)), 32, 112, 8, 5
    x = torch.randn(N * T * H * H, 16, device=dev).to(torch.bfloat16)
    dy = torch.randn(N * T * H * H, cout, device=dev).to(torch.bfloat16)
    res = {}
    arms = {"0": ("0", "0"), "1": ("1", "0"), "2": ("1", "1")}   # (stem_roll, stem_async)
    for roll in ("0", "1", "2", "0", "1", "2"):
        os.environ["PVA_ARMS"] = "stem_roll=%s,stem_async=%s" % arms[roll]
        acc = torch.zeros(cout * kt * 256, device=dev)
        C.stem_wgrad(x, dy, acc, [N, T, H, H], cout, kt)   # warm-up (and the result)
        torch.cuda.synchronize()
        out = acc.clone()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            C.stem_wgrad(x, dy, acc, [N, T, H, H], cout, kt)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        res.setdefault(roll, []).append(ms)
        res["out" + roll] = out
        print(f"stem_roll={arms[roll][0]} stem_async={arms[roll][1]}: {ms * 1000:.0f} us", flush=True)
    for k in ("1", "2"):
        a, b = res["out" + k], res["out0"]
        print(f"rel diff {arms[k]} vs {arms['0']}: {float((a - b).norm() / b.norm()):.2e}")
    # slow stem (k(1,7,7), Cout 64, 8 frames): intrinsic vs asm transpose reads
    del x, dy
    Ts, cs = 8, 64
    x = torch.randn(N * Ts * H * H, 16, device=dev).to(torch.bfloat16)
    dy = torch.randn(N * Ts * H * H, cs, device=dev).to(torch.bfloat16)
    outs = {}
    for asy in ("0", "1", "0", "1"):
        os.environ["PVA_ARMS"] = f"stem_async={asy}"
        acc = torch.zeros(cs * 256, device=dev)
        C.stem_wgrad(x, dy, acc, [N, Ts, H, H], cs, 1)
        torch.cuda.synchronize()
        outs[asy] = acc.clone()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            C.stem_wgrad(x, dy, acc, [N, Ts, H, H], cs, 1)
        e1.record()
        torch.cuda.synchronize()
        print(f"slow stem stem_async={asy}: {e0.elapsed_time(e1) / 10 * 1000:.0f} us", flush=True)
    print(f"slow stem rel diff: {float((outs['1'] - outs['0']).norm() / outs['0'].norm()):.2e}")


if __name__ == "__main__":
    main()
