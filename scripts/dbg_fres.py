import sys, torch
sys.path.insert(0, '/root/repo')
sys.path.insert(0, '/root/repo/tests')
from pytorchvideo_accelerate_amd.ops._ext import require
from pytorchvideo_accelerate_amd.ops.conv import ConvSpec, fwd_geometry, pack_weight
C = require(); DEV = torch.device('cuda')
for (N, T, H, W), c, Co, identity in [((2, 2, 8, 8), 64, 256, True), ((2, 2, 8, 8), 64, 256, False), ((2, 1, 7, 7), 16, 64, True)]:
    M = N * T * H * W
    g = torch.Generator().manual_seed(Co + identity)
    spec = ConvSpec(c, Co, (1, 1, 1))
    w = torch.randn(Co, c, 1, 1, 1, generator=g) * (2.0 / c) ** 0.5
    wf, _ = pack_weight(w.to(DEV), spec)
    yb = torch.randn(M, c, generator=g).to(torch.bfloat16).to(DEV)
    sb = (torch.rand(c, generator=g) + 0.5).to(DEV); hb = (torch.randn(c, generator=g) * 0.3).to(DEV)
    a = torch.relu(yb.float() * sb + hb).to(torch.bfloat16).double()
    fsc = (torch.rand(Co, generator=g) + 0.5).to(DEV); fsh = (torch.randn(Co, generator=g) * 0.2).to(DEV)
    resbuf = torch.randn(M, Co + 32, generator=g).to(torch.bfloat16).to(DEV); res = resbuf[:, :Co]
    rsc = None if identity else (torch.rand(Co, generator=g) + 0.5).to(DEV)
    rsh = None if identity else (torch.randn(Co, generator=g) * 0.2).to(DEV)
    yc = a @ w.view(Co, c).to(torch.bfloat16).double().t().to(DEV)
    r = res.double() if identity else res.double() * rsc.double() + rsh.double()
    ref = torch.relu(yc * fsc.double() + fsh.double() + r)
    geo = fwd_geometry(spec, N, T, H, W, c, Co + 16)
    outbuf = torch.zeros(M, Co + 16, dtype=torch.bfloat16, device=DEV); out = outbuf[:, :Co]
    mask = torch.zeros(M, Co // 8, dtype=torch.uint8, device=DEV)
    C.conv_igemm_fres(yb, wf, out, sb, hb, 2, list(geo), 8, 528, fsc, fsh, res, res.stride(0), rsc, rsh, mask)
    torch.cuda.synchronize()
    err = (out.double() - ref).abs() > 0.02 * (ref.abs() + 0.05)
    print(identity, Co, 'bad', int(err.sum()), 'of', err.numel())
    rows = err.any(1).nonzero().flatten()[:20].tolist(); cols = err.any(0).nonzero().flatten()[:40].tolist()
    print(' rows', rows); print(' cols', cols)
    if rows:
        i = rows[0]; j = err[i].nonzero().flatten()[:8].tolist()
        print(' sample', i, j, out[i, j].tolist(), ref[i, j].tolist(), (yc[i, j]*fsc[j].double()+fsh[j].double()).tolist(), r[i, j].tolist())
