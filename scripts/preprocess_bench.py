"""On-device video preprocessing (csrc/kernels/optim_pack.hip video_preprocess_kernel) at the bench shape: time
per batch and achieved HBM bandwidth.  python scripts/preprocess_bench.py [--batch 160]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchvideo_accelerate_amd.data.transforms import GpuClipBatch, sample_params  # noqa: E402
from pytorchvideo_accelerate_amd.ops._ext import require  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=160)
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--crop", type=int, default=224)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda")
    C = require()
    B, SF, H, W = a.batch, 64, 256, 340
    frames = torch.empty(B, SF, H, W, 3, dtype=torch.uint8, device=dev)
    C.synth_frames(frames, 7)
    gen = torch.Generator().manual_seed(0)
    params = [sample_params(SF, H, W, a.frames, a.crop, True, generator=gen) for _ in range(B)]
    prep = GpuClipBatch(dev, a.frames, a.crop, 4, s2d=True)
    per = SF * H * W * 3
    desc = torch.tensor([[(b * per) & 0x7FFFFFFF, (b * per) >> 31, SF, H, W, p.rh, p.rw, p.top, p.left, int(p.flip)]
                         for b, p in enumerate(params)], dtype=torch.int32, device=dev)
    tidx = torch.tensor([p.tidx for p in params], dtype=torch.int32, device=dev)
    for knob in os.environ.get("PRE_VARIANTS", "default").split(","):
        if "=" in knob:
            k, v = knob.split("=")
            os.environ[k] = v
        for _ in range(3):
            xs = prep._run(frames, desc, tidx)   # kernels only (the per-batch descriptor upload is host work)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            xs = prep._run(frames, desc, tidx)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        wr = sum(x.t.numel() * x.t.element_size() for x in xs)
        print(f"{knob}: preprocess B={B}: {ms * 1e3:.1f} us per batch, writes {wr / 1e9:.2f} GB "
              f"({wr / ms / 1e9:.2f} TB/s on the writes alone)", flush=True)


if __name__ == "__main__":
    main()
