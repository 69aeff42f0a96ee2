"""Per-op GPU time of one SlowFast training step through the fused executor (event marks).

    python scripts/layer_profile.py --batch 32 > gpurun_out/layers.txt
Prints every op (label, ms) in execution order, then totals per op kind and per pathway."""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--crop", type=int, default=224)
    a = ap.parse_args()
    from pytorchvideo_accelerate_amd.models import reference as R
    from pytorchvideo_accelerate_amd.models.fused import FusedNet
    from pytorchvideo_accelerate_amd.ops.optim import FusedSGD
    from pytorchvideo_accelerate_amd.data.transforms import GpuClipBatch, sample_params
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    T, S = a.frames, a.crop
    eng = FusedNet(R.create_slowfast(a.depth, 400, head_pool_kernel_sizes=((T // 4, S // 32, S // 32), (T, S // 32, S // 32))), dev)
    opt = FusedSGD(eng.flat, lr=0.1, momentum=0.9, weight_decay=1e-4, after_step=eng.pack)
    B = a.batch
    src_t = 2 * T
    frames = torch.empty(B, src_t, 256 if S <= 256 else S, 340 if S <= 256 else S * 4 // 3, 3, dtype=torch.uint8,
                         device=dev)
    eng.C.synth_frames(frames, 1)
    prep = GpuClipBatch(dev, T, S, 4, s2d=eng.input_s2d)
    g = torch.Generator().manual_seed(0)
    labels = torch.randint(0, 400, (B,), generator=g).to(dev)
    rows = None
    for it in range(a.steps + 1):
        xs = prep(frames, [sample_params(src_t, frames.shape[2], frames.shape[3], T, S, True, generator=g)
                           for _ in range(B)])
        opt.zero_grad()
        if it == a.steps:
            eng.prof = []
        eng.forward_backward(xs, labels)
        eng.mark("sgd+pack")
        opt.step()
        eng.mark("end")
        if it == a.steps:
            rows = eng.profile_report()
            eng.prof = None
    total = sum(ms for _, ms in rows)
    print(f"# batch {B}: step {total:.2f} ms")
    for lab, ms in rows:
        print(f"{lab:28s} {ms * 1000:9.1f} us")
    kinds = collections.defaultdict(float)
    paths = collections.defaultdict(float)
    for lab, ms in rows:
        kinds[lab.rsplit(".", 1)[-1]] += ms
        parts = lab.split(".")
        paths[parts[1] if len(parts) > 2 and parts[1] in ("p0", "p1", "fuse") else "other"] += ms
    print("\n# per op kind (ms)")
    for k, v in sorted(kinds.items(), key=lambda kv: -kv[1]):
        print(f"{k:12s} {v:8.2f}  {100 * v / total:5.1f}%")
    print("\n# per pathway (ms)")
    for k, v in sorted(paths.items(), key=lambda kv: -kv[1]):
        print(f"{k:12s} {v:8.2f}  {100 * v / total:5.1f}%")


if __name__ == "__main__":
    main()
