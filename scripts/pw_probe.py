"""Bandwidth probe of the streaming pointwise conv kernel against plain copies (M = 4M rows).

    python scripts/pw_probe.py
Prints achieved TB/s of: torch copy, a 16-B/lane HIP elementwise kernel (bn_act), and the pointwise kernel's
plain / stats / fres / backward-BN epilogues at the slow res2 shape (K = 64 -> N = 256)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    from pytorchvideo_accelerate_amd.ops._ext import require
    from pytorchvideo_accelerate_amd.ops.conv import ConvSpec, dgrad_phases, fwd_geometry, pack_weight
    from pytorchvideo_accelerate_amd.ops.tune import EXPLICIT, PW
    C = require()
    dev = torch.device("cuda")
    M, K, N = 160 * 8 * 56 * 56, 64, 256
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    res = torch.randn(M, N, device=dev).to(torch.bfloat16)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    big = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    spec = ConvSpec(K, N, (1, 1, 1))
    wf, wd = pack_weight(torch.randn(N, K, 1, 1, 1, device=dev) * 0.1, spec)
    sc, sh = torch.ones(N, device=dev), torch.zeros(N, device=dev)
    ksc, ksh = torch.ones(K, device=dev), torch.zeros(K, device=dev)
    mask = torch.empty(M, N // 8, dtype=torch.uint8, device=dev)
    geo = list(fwd_geometry(spec, 1, 1, M, 1, K, N))
    rows = []

    def rep(name, t, nbytes):
        rows.append((name, t * 1e6, nbytes / t / 1e12))
        print("%-40s %8.1f us %6.2f TB/s" % rows[-1], flush=True)

    rep("torch copy [M,256]", timeit(lambda: big.copy_(res)), 2 * res.numel() * 2)
    for v in (0, 1, 2, 4, 5, 6):
        cfg = EXPLICIT | PW | v
        r = C.conv_cfg_bm(cfg, N)
        stats = torch.empty((M + r - 1) // r, 2, N, device=dev)
        rep("pw%d%s plain" % (r, "s" * (v >> 2)), timeit(lambda: C.conv_igemm(x, wf, out, None, None, None, 0, 0, geo, 8, cfg)),
            (x.numel() + out.numel()) * 2)
        rep("pw%d%s stats+affine" % (r, "s" * (v >> 2)), timeit(lambda: C.conv_igemm(x, wf, out, stats, ksc, ksh, 2, 0, geo, 8, cfg)),
            (x.numel() + out.numel()) * 2)
        rep("pw%d%s fres" % (r, "s" * (v >> 2)), timeit(lambda: C.conv_igemm_fres(x, wf, out, ksc, ksh, 2, geo, 8, cfg, sc, sh, res, N,
                                                             None, None, mask)),
            (x.numel() + out.numel() + res.numel()) * 2 + mask.numel())
    # backward-BN epilogue: conv_a dgrad of res2 (dy [M,64] -> dx [M,256]) with residual, mask, partials
    dy = x
    dgeo = list(dgrad_phases(ConvSpec(N, K, (1, 1, 1)), 1, (1, M, 1), (1, M, 1), K, N)[0])
    _, wd2 = pack_weight(torch.randn(K, N, 1, 1, 1, device=dev) * 0.1, ConvSpec(N, K, (1, 1, 1)))
    for v in (0, 1, 2, 4, 5, 6):
        cfg = EXPLICIT | PW | v
        r = C.conv_cfg_bm(cfg, N)
        part = torch.empty((M + r - 1) // r, 3, N, device=dev)
        rep("pw%d%s dgrad res+mask+part" % (r, "s" * (v >> 2)),
            timeit(lambda: C.conv_igemm_epi(dy, wd2, out, 0, dgeo, 8, res, N, mask, None, None, None, None, None,
                                            None, part, None, None, cfg)),
            (dy.numel() + out.numel() + res.numel()) * 2 + mask.numel())
    # backward-BN epilogue with the producer's BN input (conv_c dgrad of res2: dy [M,256] -> [M,64], ReLU mask
    # from affine(y_b), partial sums of sum(dz), sum(dz y_b))
    cgeo = list(dgrad_phases(ConvSpec(K, N, (1, 1, 1)), 1, (1, M, 1), (1, M, 1), N, K)[0])
    _, wdc = pack_weight(torch.randn(N, K, 1, 1, 1, device=dev) * 0.1, ConvSpec(K, N, (1, 1, 1)))
    dyc = res
    yb = torch.randn(M, K, device=dev).to(torch.bfloat16)
    outk = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    mk, rk = torch.zeros(K, device=dev), torch.ones(K, device=dev)
    for v in (0, 1, 2, 4, 5, 6):
        cfg = EXPLICIT | PW | v
        r = C.conv_cfg_bm(cfg, K)
        part = torch.empty((M + r - 1) // r, 3, K, device=dev)
        rep("pw%d%s dgrad bn(y0)+part K=256" % (r, "s" * (v >> 2)),
            timeit(lambda: C.conv_igemm_epi(dyc, wdc, outk, 0, cgeo, 8, None, 0, None, yb, mk, rk, None, None,
                                            None, part, ksc, ksh, cfg)),
            (dyc.numel() + outk.numel() + yb.numel()) * 2)
    # BN-backward apply (dy = A dz*mask + B y + C) at the same shape: reads g, y, mask bits; writes dy
    y = res
    coef = torch.randn(3 * N, device=dev)
    mbits = torch.randint(0, 255, (M, N // 8), dtype=torch.uint8, device=dev)
    rep("bn_bwd_apply [M,256] mask bits",
        timeit(lambda: C.bn_bwd_apply(out, N, 3, mbits, N // 8, None, None, y, coef, big, None, None, None, None, 0,
                                      0, M, N)),
        3 * out.numel() * 2 + mbits.numel())
    for cfg in (-1,):
        rep("igemm heuristic plain", timeit(lambda: C.conv_igemm(x, wf, out, None, None, None, 0, 0, geo, 8, cfg)),
            (x.numel() + out.numel()) * 2)


if __name__ == "__main__":
    main()
