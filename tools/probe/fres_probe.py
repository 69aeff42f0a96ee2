import os, sys, torch
sys.path.insert(0, "/root/repo")
from pytorchvideo_accelerate_amd.ops._ext import require
from pytorchvideo_accelerate_amd.ops.conv import ConvSpec, fwd_geometry
from pytorchvideo_accelerate_amd.ops.tune import EXPLICIT, PW, PW_SOLO, PW_W4
C = require(); dev = torch.device("cuda"); bf = torch.bfloat16
N, T, H, W, CI, CO = 160, 8, 56, 56, 64, 256
M = N * T * H * W
yb = torch.randn(M, CI, device=dev).to(bf); w = (torch.randn(CO, CI, device=dev) * 0.1).to(bf)
out = torch.empty(M, CO, device=dev, dtype=bf); res = torch.randn(M, CO, device=dev).to(bf)
mask = torch.empty(M, CO // 8, device=dev, dtype=torch.uint8)
sc = torch.rand(CI, device=dev); sh = torch.randn(CI, device=dev) * 0.1
osc = torch.rand(CO, device=dev); osh = torch.randn(CO, device=dev) * 0.1
g = fwd_geometry(ConvSpec(CI, CO, (1, 1, 1), (1, 1, 1), (0, 0, 0)), N, T, H, W, CI, CO)
for probe in ("1", "0"):
    os.environ["PVA_PW_NT"] = probe
    for cfg in (EXPLICIT | PW | 2, EXPLICIT | PW | 2 | PW_SOLO, EXPLICIT | PW | 0):
        f = lambda: C.conv_igemm_fres(yb, w, out, sc, sh, 2, g, 8, cfg, osc, osh, res, CO, None, None, mask)
        for _ in range(3): f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10): f()
        e1.record(); torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 10 * 1e3
        print(f"probe {probe} cfg {cfg}: {us:.1f} us", flush=True)
