"""Sensitivity of the SlowFast-R50 training gradient at random init to tiny perturbations, on the PyTorch modules
in fp32 (no fused kernels): the cosine between the flat parameter gradients of (x, y) and of (x * (1 + eps*n), y)
for eps = 1e-6 / 1e-4 / 1e-2, and between fp32 and bf16-autocast gradients of the same input.  A cosine far below
1 at eps ~ bf16 rounding means run-to-run gradient differences of the fused executor's non-deterministic mode
(fp32-atomic reductions) are the network's own chaos, not an executor error."""
import os
import sys

import torch
import torch.nn.functional as F

os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from pytorchvideo_accelerate_amd.models import reference as R
    B = int(os.environ.get("B", "4"))
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = R.create_slowfast(50, 400, dropout_rate=0.0).to(dev).train()
    g = torch.Generator().manual_seed(1)
    fast = torch.randn(B, 3, 32, 224, 224, generator=g).to(dev)
    y = torch.randint(0, 400, (B,), generator=g).to(dev)
    noise = torch.randn(fast.shape, generator=torch.Generator().manual_seed(2)).to(dev)
    state = {k: v.clone() for k, v in m.state_dict().items()}

    def grad(x, ac=False):
        m.load_state_dict(state)   # identical BN running stats each call
        m.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=ac):
            out = m([x[:, :, ::4].contiguous(), x])
        F.cross_entropy(out.float(), y).backward()
        return torch.cat([p.grad.reshape(-1).float() for p in m.parameters()])

    g0 = grad(fast)
    for eps in (1e-6, 1e-4, 1e-2):
        g1 = grad(fast * (1 + eps * noise))
        print("eps %.0e: cos %.5f rel %.3e" % (eps, float(F.cosine_similarity(g0, g1, dim=0)),
                                                float((g1 - g0).norm() / g0.norm())), flush=True)
    ga = grad(fast, ac=True)
    print("autocast vs fp32: cos %.5f rel %.3e" % (float(F.cosine_similarity(g0, ga, dim=0)),
                                                   float((ga - g0).norm() / g0.norm())), flush=True)


if __name__ == "__main__":
    main()
