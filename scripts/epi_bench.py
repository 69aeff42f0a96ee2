"""Microbenchmark of the dgrad backward-BN epilogue: which feature costs what (res2-slow / res4 shapes)."""
import sys, os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchvideo_accelerate_amd.ops._ext import require
from pytorchvideo_accelerate_amd.ops.conv import Act, ConvSpec, conv_m_tiles, dgrad_phases, pack_weight

C = require()
DEV = "cuda"


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1000


for (cin, cout, k, pad, dims) in [(256, 64, (1, 1, 1), (0, 0, 0), (32, 8, 56, 56)),
                                  (1024, 256, (3, 1, 1), (1, 0, 0), (32, 8, 14, 14)),
                                  (32, 8, (3, 1, 1), (1, 0, 0), (32, 32, 56, 56))]:
    N, T, H, W = dims
    spec = ConvSpec(cin, cout, k, (1, 1, 1), pad)
    w = torch.randn(cout, cin, *k, device=DEV) * 0.05
    _, wd = pack_weight(w, spec)
    M = N * T * H * W
    dy = Act(torch.randn(M, cout, device=DEV).to(torch.bfloat16), N, T, H, W)
    out = torch.empty(M, cin, device=DEV, dtype=torch.bfloat16)
    res = torch.randn(M, cin, device=DEV).to(torch.bfloat16)
    y0 = torch.randn(M, cin, device=DEV).to(torch.bfloat16)
    y1 = torch.randn(M, cin, device=DEV).to(torch.bfloat16)
    mask = torch.randint(0, 255, (M, cin // 8), device=DEV, dtype=torch.uint8)
    mu, rs = torch.zeros(cin, device=DEV), torch.ones(cin, device=DEV)
    g = dgrad_phases(spec, N, (T, H, W), (T, H, W), cout, cin)[0]
    tiles = conv_m_tiles(M, cin)
    part = torch.empty(tiles * 3 * cin, device=DEV)
    mb = M * cin * 2 / 1e6
    print(f"== dgrad M={M} Cin={cin} K={cout * k[0]}  (one [M,Cin] bf16 tensor = {mb:.0f} MB)")
    cases = {
        "plain": lambda: C.conv_igemm(dy.t, wd, out, None, None, None, 0, 0, g, 8),
        "plain+accum": lambda: C.conv_igemm(dy.t, wd, out, None, None, None, 0, 1, g, 8),
        "epi mask": lambda: C.conv_igemm_epi(dy.t, wd, out, 0, g, 8, None, 0, mask, None, None, None, None, None, None, None),
        "epi res": lambda: C.conv_igemm_epi(dy.t, wd, out, 0, g, 8, res, cin, None, None, None, None, None, None, None, None),
        "epi stats": lambda: C.conv_igemm_epi(dy.t, wd, out, 0, g, 8, None, 0, None, y0, mu, rs, None, None, None, part),
        "epi res+mask+stats": lambda: C.conv_igemm_epi(dy.t, wd, out, 0, g, 8, res, cin, mask, y0, mu, rs, None, None, None, part),
        "epi all+dual": lambda: C.conv_igemm_epi(dy.t, wd, out, 0, g, 8, res, cin, mask, y0, mu, rs, y1, mu, rs, part),
    }
    for name, fn in cases.items():
        print(f"  {name:22s} {bench(fn):8.1f} us", flush=True)

