"""Multi-workgroup numerics / determinism check of the pointwise kernel (M spans many row blocks, with a
partial last tile): forward plain+stats+affine, fres, and the dgrad backward-BN epilogue, each run twice
and compared bitwise and against a float reference."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from pytorchvideo_accelerate_amd.ops._ext import require
    from pytorchvideo_accelerate_amd.ops.conv import ConvSpec, fwd_geometry, pack_weight
    from pytorchvideo_accelerate_amd.ops.tune import EXPLICIT, PW, PW_SOLO
    C = require()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for M, K, N in [(100003, 64, 256), (70001, 8, 32), (50017, 16, 64), (40009, 256, 64), (30011, 128, 512)]:
        spec = ConvSpec(K, N, (1, 1, 1))
        w = torch.randn(N, K, 1, 1, 1, device=dev, generator=g) * (2.0 / K) ** 0.5
        wf, _ = pack_weight(w, spec)
        x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        sc = torch.rand(K, device=dev, generator=g) + 0.5
        sh = torch.randn(K, device=dev, generator=g) * 0.3
        a = torch.relu(x.float() * sc + sh).to(torch.bfloat16).float()
        ref = a @ w.view(N, K).to(torch.bfloat16).float().t()
        geo = list(fwd_geometry(spec, 1, 1, M, 1, K, N))
        for cfg in (EXPLICIT | PW, EXPLICIT | PW | 2, EXPLICIT | PW | PW_SOLO):
            r = C.conv_cfg_bm(cfg, N)
            outs = []
            for rep in range(2):
                out = torch.full((M, N), float("nan"), device=dev).to(torch.bfloat16)
                stats = torch.zeros((M + r - 1) // r, 2, N, device=dev)
                C.conv_igemm(x, wf, out, stats, sc, sh, 2, 0, geo, 8, cfg)
                torch.cuda.synchronize()
                outs.append((out, stats.sum(0)))
            o0, s0 = outs[0]
            o1, s1 = outs[1]
            err = ((o0.float() - ref).norm() / ref.norm()).item()
            rs = o0.float()
            serr = ((s0[0] - rs.sum(0)).norm() / rs.sum(0).norm()).item()
            print("M=%d K=%d N=%d cfg=%d: rel %.2e stats %.2e det %s nan %d" % (
                M, K, N, cfg, err, serr, torch.equal(o0, o1), int(torch.isnan(o0.float()).sum())), flush=True)


if __name__ == "__main__":
    main()


def backward_and_fres():
    from pytorchvideo_accelerate_amd.ops._ext import require
    from pytorchvideo_accelerate_amd.ops.conv import ConvSpec, dgrad_phases, fwd_geometry, pack_weight
    from pytorchvideo_accelerate_amd.ops.tune import EXPLICIT, PW, PW_SOLO
    C = require()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(1)
    for M, K, N in [(100003, 64, 256), (70001, 8, 32), (40009, 256, 64)]:
        # fres: out = relu(fsc * (relu(x sc + sh) W^T) + fsh + res)
        spec = ConvSpec(K, N, (1, 1, 1))
        w = torch.randn(N, K, 1, 1, 1, device=dev, generator=g) * (2.0 / K) ** 0.5
        wf, _ = pack_weight(w, spec)
        x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        sc = torch.rand(K, device=dev, generator=g) + 0.5
        sh = torch.randn(K, device=dev, generator=g) * 0.3
        fsc = torch.rand(N, device=dev, generator=g) + 0.5
        fsh = torch.randn(N, device=dev, generator=g) * 0.2
        res = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
        a = torch.relu(x.float() * sc + sh).to(torch.bfloat16).float()
        ref = torch.relu((a @ w.view(N, K).to(torch.bfloat16).float().t()) * fsc + fsh + res.float())
        geo = list(fwd_geometry(spec, 1, 1, M, 1, K, N))
        for cfg in (EXPLICIT | PW, EXPLICIT | PW | 2):
            outs = []
            for rep in range(2):
                out = torch.full((M, N), float("nan"), device=dev).to(torch.bfloat16)
                mask = torch.zeros(M, N // 8, dtype=torch.uint8, device=dev)
                C.conv_igemm_fres(x, wf, out, sc, sh, 2, geo, 8, cfg, fsc, fsh, res, N, None, None, mask)
                torch.cuda.synchronize()
                outs.append((out, mask))
            err = ((outs[0][0].float() - ref).norm() / ref.norm()).item()
            print("fres M=%d K=%d N=%d cfg=%d: rel %.2e det %s/%s" % (M, K, N, cfg, err, torch.equal(outs[0][0], outs[1][0]),
                                                                 torch.equal(outs[0][1], outs[1][1])), flush=True)
        # dgrad epilogue: dx = (dy W) + res, masked by bits; partial sums
        dspec = ConvSpec(N, K, (1, 1, 1))   # conv N -> K, its dgrad maps dy [M,K] -> dx [M,N]
        dgeo = list(dgrad_phases(dspec, 1, (1, M, 1), (1, M, 1), K, N)[0])
        wd_src = torch.randn(K, N, 1, 1, 1, device=dev, generator=g) * 0.1
        _, wd = pack_weight(wd_src, dspec)
        dy = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        bits = torch.randint(0, 256, (M, N // 8), dtype=torch.uint8, device=dev, generator=g)
        mk = ((bits.unsqueeze(-1).int() >> torch.arange(8, device=dev)) & 1).view(M, N).bool()
        dref = (dy.float() @ wd_src.view(K, N).to(torch.bfloat16).float() + res.float()) * mk
        for cfg in (EXPLICIT | PW, EXPLICIT | PW | 2):
            r = C.conv_cfg_bm(cfg, N)
            outs = []
            for rep in range(2):
                out = torch.full((M, N), float("nan"), device=dev).to(torch.bfloat16)
                part = torch.zeros((M + r - 1) // r, 3, N, device=dev)
                C.conv_igemm_epi(dy, wd, out, 0, dgeo, 8, res, N, bits, None, None, None, None, None, None, part,
                                 None, None, cfg)
                torch.cuda.synchronize()
                outs.append((out, part.sum(0)))
            o = outs[0][0].float()
            err = ((o - dref).norm() / dref.norm()).item()
            serr = ((outs[0][1][0] - o.sum(0)).norm() / o.sum(0).norm()).item()
            print("dgrad M=%d K=%d N=%d cfg=%d: rel %.2e part %.2e det %s" % (M, K, N, cfg, err, serr,
                                                                          torch.equal(outs[0][0], outs[1][0])), flush=True)


if __name__ == "__main__":
    backward_and_fres()
