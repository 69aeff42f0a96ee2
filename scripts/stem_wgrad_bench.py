"""Fast-stem weight gradient at the headline shape (SlowFast-R50 32x2x224, B=160: s2d input [160, 32, 112, 112, 16],
dY [.., 8]), the rolling-fragment frame-pair kernel (default) against the one-tap-row-per-wave form
(PVA_STEM_ROLL=0, read per launch).  Prints the mean kernel time of each and their results' relative difference."""
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
    for roll in ("0", "1", "0", "1"):
        os.environ["PVA_STEM_ROLL"] = roll
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
        print(f"PVA_STEM_ROLL={roll}: {ms * 1000:.0f} us", flush=True)
    a, b = res["out0"], res["out1"]
    print(f"rel diff roll vs no-roll: {float((a - b).norm() / b.norm()):.2e}")


if __name__ == "__main__":
    main()
