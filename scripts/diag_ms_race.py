"""Gradient reproducibility of FusedNet.forward_backward across the single- and two-stream schedules at the
real SlowFast-R50 32x2x224 shape and a small batch (dropout off, same inputs every call): relative L2
difference of the flat gradient between repeated calls.  Atomics give ~1e-6; anything larger is a race."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from pytorchvideo_accelerate_amd.models import reference as R
    from pytorchvideo_accelerate_amd.models.fused import FusedNet
    B = int(os.environ.get("B", "4"))
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = R.create_slowfast(50, 400)
    model.blocks[-1].dropout.p = 0.0
    eng = FusedNet(model, dev, deterministic=os.environ.get("DET", "0") == "1")
    g = torch.Generator().manual_seed(1)
    fast = torch.randn(B, 3, 32, 224, 224, generator=g)
    slow = fast[:, :, ::4].contiguous()
    acts = eng.prepare_inputs([slow, fast])
    labels = torch.randint(0, 400, (B,), generator=g).to(dev)
    eng.forward_backward(acts, labels, accumulate=False)   # tuning step (single stream)
    torch.cuda.synchronize()
    grads = {}
    for tag, ms in (("s0", False), ("s1", False), ("m0", True), ("m1", True), ("m2", True), ("s2", False)):
        eng._ms_ok = ms
        loss, _ = eng.forward_backward(acts, labels, accumulate=False)
        torch.cuda.synchronize()
        grads[tag] = eng.flat.grad.clone()
        print(tag, "loss %.6f |g| %.6e" % (float(loss), float(grads[tag].norm())), flush=True)
    ref = grads["s0"]
    conv = torch.zeros_like(ref, dtype=torch.bool)
    for nm, p in zip(eng.flat.names, eng.flat.params):
        a, b = eng.flat.span(p)
        if nm.endswith(".w") and not nm.endswith("bn.w"):
            conv[a:b] = True
    print("share of |g|^2 in conv weights %.3f" % float(ref[conv].norm() ** 2 / ref.norm() ** 2), flush=True)
    for tag, gg in grads.items():
        d = (gg - ref)
        rel = float(d.norm() / ref.norm())
        print("%s vs s0: rel %.3e  conv-weights rel %.3e  cos %.5f" % (
            tag, rel, float(d[conv].norm() / ref[conv].norm()),
            float(torch.nn.functional.cosine_similarity(gg, ref, dim=0))), flush=True)
        if rel > 1e-4:
            # worst parameters
            worst = []
            for nm, p in zip(eng.flat.names, eng.flat.params):
                a, b = eng.flat.span(p)
                worst.append((float(d[a:b].norm() / (ref[a:b].norm() + 1e-30)), nm))
            worst.sort(reverse=True)
            for r, nm in worst[:12]:
                print("   %-28s rel %.3e" % (nm, r), flush=True)


if __name__ == "__main__":
    main()
