"""Diagnostic: per-32-channel-chunk error of the pointwise conv kernel for one forward case."""
import sys
import os
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from pytorchvideo_accelerate_amd.ops._ext import require
from pytorchvideo_accelerate_amd.ops.conv import ConvSpec, fwd_geometry, pack_weight
from pytorchvideo_accelerate_amd.ops.tune import EXPLICIT, PW

C = require()
DEV = torch.device("cuda")
for (N_, T, H, W), ci, co, aff in [((1, 4, 10, 10), 128, 512, 1), ((1, 4, 10, 10), 128, 512, 0),
                                   ((1, 4, 10, 10), 128, 512, 2)]:
    M = N_ * T * H * W
    g = torch.Generator().manual_seed(0)
    spec = ConvSpec(ci, co, (1, 1, 1))
    w = torch.randn(co, ci, 1, 1, 1, generator=g) * 0.1
    wf, _ = pack_weight(w.to(DEV), spec)
    x = torch.randn(M, ci, generator=g).to(torch.bfloat16).to(DEV)
    sc = (torch.rand(ci, generator=g) + 0.5).to(DEV)
    sh = (torch.randn(ci, generator=g) * 0.3).to(DEV)
    xin = x.double()
    if aff:
        xin = x.float() * sc + sh
        xin = (torch.relu(xin) if aff == 2 else xin).to(torch.bfloat16).double()
    ref = xin @ w.view(co, ci).to(torch.bfloat16).double().t().to(DEV)
    geo = list(fwd_geometry(spec, N_, T, H, W, ci, co))
    y = torch.full((M, co), 7.0, dtype=torch.bfloat16, device=DEV)
    C.conv_igemm(x, wf, y, None, sc if aff else None, sh if aff else None, aff, 0, geo, 8, EXPLICIT | PW)
    torch.cuda.synchronize()
    err = ((y.double() - ref).abs().view(M, co // 32, 32).amax(dim=(0, 2)))
    print("aff", aff, "max err per chunk", [round(v, 3) for v in err.tolist()])
    print("  y[0,:8]", y[0, :8].tolist(), "ref", [round(v, 3) for v in ref[0, :8].tolist()])
