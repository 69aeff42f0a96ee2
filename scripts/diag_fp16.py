"""fp16 range diagnostic: one fused fp16 training step at several loss scales; lists the parameters whose gradient is
non-finite and every fp16 workspace tensor (activations / gradients, folded weights) that holds an inf or nan, with
its max |finite| value — locates where an overflow starts.

    python scripts/diag_fp16.py [--scales 8 12 16] [--size 64 --frames 8 --batch 2]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchvideo_accelerate_amd.models import reference as R  # noqa: E402
from pytorchvideo_accelerate_amd.models.fused import FusedNet  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scales", type=int, nargs="+", default=[8, 12, 16])
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--batch", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda")
    for e in a.scales:
        torch.manual_seed(0)
        if a.size == 64:
            model = R.create_slowfast(50, 10, head_pool_kernel_sizes=((2, 2, 2), (8, 2, 2)), dropout_rate=0.0)
        else:
            model = R.create_slowfast(50, 400, dropout_rate=0.0)
        eng = FusedNet(model, dev, compute_dtype=torch.float16)
        g = torch.Generator().manual_seed(3)
        fast = torch.randn(a.batch, 3, a.frames, a.size, a.size, generator=g).half().float()
        idx = torch.linspace(0, a.frames - 1, a.frames // 4).long()
        xs = eng.prepare_inputs([fast[:, :, idx].contiguous(), fast])
        labels = torch.arange(a.batch, device=dev) % 10
        loss, _ = eng.forward_backward(xs, labels, loss_scale=2.0 ** e)
        torch.cuda.synchronize()
        bad = [n for n, p in model.named_parameters() if not torch.isfinite(p.grad).all()]
        print(f"== loss scale 2^{e}: loss {float(loss):.4f}; {len(bad)} non-finite parameter gradients", flush=True)
        for n in bad[:12]:
            print("   grad", n)
        items = list(eng._ws.items())
        for u in eng.units:
            for nm in ("W1t", "W2"):
                t = getattr(u, nm, None)
                if t is not None:
                    items.append(((u.name, nm), t))
        for k, t in items:
            if t.dtype != torch.float16:
                continue
            f = t.float()
            fin = torch.isfinite(f)
            if not fin.all():
                mx = f[fin].abs().max().item() if fin.any() else float("nan")
                print(f"   non-finite {k}: {int((~fin).sum())} of {f.numel()} (max |finite| {mx:.4g})")


if __name__ == "__main__":
    main()
