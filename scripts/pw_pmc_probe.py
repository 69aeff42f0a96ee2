"""Tiny driver for PMC passes over the pointwise kernel's streaming epilogues (scripts/gpu_r2_pwpmc.sh):
one kernel per op so a per-kernel-name summary separates them — a torch copy, bn_bwd_apply, the pointwise
plain epilogue and its backward-BN epilogue (residual + mask bits + partials) at the slow res2 shape."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from pytorchvideo_accelerate_amd.ops._ext import require
    from pytorchvideo_accelerate_amd.ops.conv import ConvSpec, dgrad_phases, fwd_geometry, pack_weight
    from pytorchvideo_accelerate_amd.ops.tune import EXPLICIT, PW, PW_SOLO
    C = require()
    dev = torch.device("cuda")
    M, K, N = 160 * 8 * 56 * 56, 64, 256
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    res = torch.randn(M, N, device=dev).to(torch.bfloat16)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    big = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    spec = ConvSpec(K, N, (1, 1, 1))
    wf, _ = pack_weight(torch.randn(N, K, 1, 1, 1, device=dev) * 0.1, spec)
    geo = list(fwd_geometry(spec, 1, 1, M, 1, K, N))
    mask = torch.randint(0, 255, (M, N // 8), dtype=torch.uint8, device=dev)
    dgeo = list(dgrad_phases(ConvSpec(N, K, (1, 1, 1)), 1, (1, M, 1), (1, M, 1), K, N)[0])
    _, wd2 = pack_weight(torch.randn(K, N, 1, 1, 1, device=dev) * 0.1, ConvSpec(N, K, (1, 1, 1)))
    cfg_d = EXPLICIT | PW | 2
    part = torch.empty((M + 4095) // 4096, 3, N, device=dev)
    coef = torch.randn(3 * N, device=dev)
    ops = [
        ("copy", lambda: big.copy_(res)),
        ("bn_bwd_apply", lambda: C.bn_bwd_apply(out, N, 3, mask, N // 8, None, None, res, coef, big, None, None,
                                                None, None, 0, 0, M, N)),
        ("pw plain", lambda: C.conv_igemm(x, wf, out, None, None, None, 0, 0, geo, 8, EXPLICIT | PW | PW_SOLO)),
        ("pw dgrad res", lambda: C.conv_igemm_epi(x, wd2, out, 0, dgeo, 8, res, N, mask, None, None, None, None,
                                                  None, None, part, None, None, cfg_d)),
    ]
    for name, fn in ops:
        for _ in range(4):
            fn()
        torch.cuda.synchronize()
        print(name, "done", flush=True)


if __name__ == "__main__":
    main()
