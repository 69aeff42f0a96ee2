"""Stock PyTorch-ROCm eager baseline (BASELINE.md protocol).

Same model / config / synthetic data as bench.py but every op is the stock
PyTorch path (MIOpen conv3d, ATen BN/ReLU/pool, foreach SGD) under bf16 autocast.

    python scripts/baseline_torch.py --batch 8 --steps 20 --warmup 5 [--channels-last]
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchvideo_accelerate_amd.models.reference import create_slowfast, slow_r50  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--crop", type=int, default=224)
    ap.add_argument("--alpha", type=int, default=4)
    ap.add_argument("--classes", type=int, default=400)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--channels-last", action="store_true")
    ap.add_argument("--slow", action="store_true")
    ap.add_argument("--dtype", default="bf16")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = (slow_r50(a.classes) if a.slow else create_slowfast(a.depth, a.classes)).to(dev)
    if a.channels_last:
        model = model.to(memory_format=torch.channels_last_3d)
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    B, T, S = a.batch, a.frames, a.crop
    fast = torch.randn(B, 3, T, S, S, device=dev)
    slow = fast[:, :, torch.linspace(0, T - 1, T // a.alpha).long().to(dev)].contiguous()
    if a.channels_last:
        fast = fast.contiguous(memory_format=torch.channels_last_3d)
        slow = slow.contiguous(memory_format=torch.channels_last_3d)
    x = fast if a.slow else [slow, fast]  # Slow-R50 takes the T-frame clip itself
    y = torch.randint(0, a.classes, (B,), device=dev)
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": None}[a.dtype]

    def step():
        with torch.autocast("cuda", dtype=dt or torch.bfloat16, enabled=dt is not None):
            out = model(x)
        loss = F.cross_entropy(out.float(), y)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    for i in range(a.warmup):
        step()
        print(f"warmup step {i}", file=sys.stderr, flush=True)   # progress (a silent minute reads as a hang)
    torch.cuda.synchronize()
    times = []
    for _ in range(a.steps):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        l = step()
        e.record()
        e.synchronize()
        times.append(s.elapsed_time(e))
        print(f"step {len(times)}: {times[-1]:.1f} ms", file=sys.stderr, flush=True)
    times.sort()
    p50 = times[len(times) // 2]
    mean = sum(times) / len(times)
    print(json.dumps({"impl": "stock_torch", "dtype": a.dtype, "slow": a.slow, "channels_last": a.channels_last, "batch": B, "frames": T, "crop": S,
                      "p50_ms": p50, "mean_ms": mean, "p90_ms": times[int(len(times) * 0.9) - 1],
                      "clips_per_s": B * 1000.0 / mean, "loss": float(l)}))


if __name__ == "__main__":
    main()
