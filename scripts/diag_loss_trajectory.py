"""Is the bench's above-chance final loss (7.0 > ln 400 = 5.99, BENCH_r05 ``final_loss``) the recipe or the kernels?

Runs the bench recipe — SlowFast-R50 32x2x224, random-init weights, SGD lr 0.1 / momentum 0.9 / wd 1e-4, random
labels over 400 classes, a fresh clip batch every step — on identical inputs and initial weights through
  * the fused bf16 executor (models/fused.FusedNet, the bench's kernels and autotuned configurations), and
  * the native fp32 executor (models/native32.NativeF32Net, ~fp32 accurate: the oracle),
and prints both loss trajectories as JSON lines.  Dropout is on in both (different Philox streams), so the
trajectories are two samples of the same recipe, not bitwise twins.

    python scripts/diag_loss_trajectory.py --batch 48 --steps 8
"""
import argparse
import copy
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=48)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--crop", type=int, default=224)
    a = ap.parse_args()
    from pytorchvideo_accelerate_amd.models import reference as R
    from pytorchvideo_accelerate_amd.models.fused import FusedNet
    from pytorchvideo_accelerate_amd.models.native32 import NativeF32Net
    from pytorchvideo_accelerate_amd.ops.optim import FusedSGD
    dev = torch.device("cuda")
    torch.manual_seed(1234)
    model = R.create_slowfast(50, 400)
    gen = torch.Generator().manual_seed(7)
    B, T, S = a.batch, a.frames, a.crop
    idx = torch.linspace(0, T - 1, T // 4).long()
    batches = []
    for _ in range(a.steps):
        fast = torch.randn(B, 3, T, S, S, generator=gen)
        batches.append(([fast[:, :, idx].contiguous(), fast], torch.randint(0, 400, (B,), generator=gen)))
    out = {}
    for name in ("fp32", "bf16"):
        m = copy.deepcopy(model)
        if name == "fp32":
            eng = NativeF32Net(m, dev)
            opt = FusedSGD(eng.flat, lr=a.lr, momentum=0.9, weight_decay=1e-4)
            prep = lambda xs: xs   # noqa: E731
        else:
            eng = FusedNet(m, dev)
            opt = FusedSGD(eng.flat, lr=a.lr, momentum=0.9, weight_decay=1e-4, after_step=eng.pack)
            prep = eng.prepare_inputs
        losses = []
        for xs, y in batches:
            opt.zero_grad()
            loss, _ = eng.forward_backward(prep(xs), y.to(dev))
            opt.step()
            losses.append(round(float(loss), 4))
            print(json.dumps({"executor": name, "step": len(losses), "loss": losses[-1]}), flush=True)
        out[name] = losses
        del eng, opt, m
        torch.cuda.empty_cache()
    print(json.dumps({"batch": B, "lr": a.lr, "ln_classes": 5.9915, **out}), flush=True)


if __name__ == "__main__":
    main()
