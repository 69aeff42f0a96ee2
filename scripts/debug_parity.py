"""Layer-by-layer comparison of the fused executor against the PyTorch oracle (diagnostic tool).

    python scripts/debug_parity.py [--slow] [--size 64] [--frames 8] [--batch 2]
"""
import argparse
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchvideo_accelerate_amd.models import reference as R  # noqa: E402
from pytorchvideo_accelerate_amd.models.fused import FusedNet  # noqa: E402


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slow", action="store_true")
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--batch", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    S, T, N = a.size, a.frames, a.batch
    hs = S // 32
    if a.slow:
        model = R.create_resnet(50, 10, head_pool_kernel_size=(1, hs, hs), dropout_rate=0.0)
    else:
        model = R.create_slowfast(50, 10, head_pool_kernel_sizes=((T // 4, hs, hs), (T, hs, hs)), dropout_rate=0.0)
    oracle = copy.deepcopy(model).to(dev).train()
    g = torch.Generator().manual_seed(0)
    fast = torch.randn(N, 3, T, S, S, generator=g).to(torch.bfloat16).float()
    xs = [fast] if a.slow else [fast[:, :, torch.linspace(0, T - 1, T // 4).long()].contiguous(), fast]
    labels = torch.arange(N, device=dev) % 10
    rec = {}

    def hook(name):
        def f(m, i, o):
            rec[name] = o.detach()
        return f

    for n, m in oracle.named_modules():
        if isinstance(m, torch.nn.Conv3d):
            m.register_forward_hook(hook(n))
    inp = [x.to(dev) for x in xs] if not a.slow else xs[0].to(dev)
    out_ref = oracle(inp)
    loss_ref = F.cross_entropy(out_ref, labels)
    loss_ref.backward()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        o2 = copy.deepcopy(model).to(dev).train()(inp)
    print("loss oracle fp32 %.5f  oracle autocast-bf16 %.5f" % (loss_ref.item(), F.cross_entropy(o2.float(), labels).item()))
    eng = FusedNet(model, dev)
    # map oracle conv names -> fused units
    conv2name = {id(m): n for n, m in model.named_modules()}
    loss, logits = eng.forward_backward(eng.prepare_inputs(xs), labels)
    torch.cuda.synchronize()
    print("loss fused %.5f" % loss.item(), "logits rel %.4f" % rel(logits, out_ref.detach()))
    for u in eng.units:
        n = conv2name[id(u.conv)]
        y = eng._ws[(u.name, "y", "t")]
        ref = rec[n]
        To, Ho, Wo = ref.shape[2:]
        yf = y.float().reshape(ref.shape[0], To, Ho, Wo, -1).permute(0, 4, 1, 2, 3)
        print(f"{u.name:14s} {n:60s} fwd rel {rel(yf, ref):.4f}")
    refp = dict(oracle.named_parameters())
    for n, p in model.named_parameters():
        print(f"grad {n:70s} {rel(p.grad, refp[n].grad):.4f}")


if __name__ == "__main__":
    main()
