"""Numerics of the narrow direct-to-register conv kernel (csrc/kernels/conv_direct.hip) against PyTorch fp32.

Every launch forces the direct configuration word (tune.EXPLICIT | tune.DIRECT [| DIRECT_2K]) so the test
exercises that kernel, not whichever configuration the autotuner would pick: forward (+consumer-side
BN-ReLU fold, +BN partial sums), strided dgrad phases (+accumulate), and the backward-BN dgrad epilogue.
"""
import pytest
import torch

from pytorchvideo_accelerate_amd.ops.conv import Act, ConvSpec, dgrad_phases, fwd_geometry, pack_weight
from pytorchvideo_accelerate_amd.ops.tune import DIRECT, DIRECT_2K, DIRECT_HALF, EXPLICIT

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (cin, cout, k, stride, pad, (N, T, H, W)) — fast-pathway / fusion classes with N (or Cin for dgrad) <= 64
CASES = [
    (8, 8, (1, 3, 3), (1, 1, 1), (0, 1, 1), (2, 8, 30, 30)),        # fast res2 conv_b
    (32, 8, (3, 1, 1), (1, 1, 1), (1, 0, 0), (2, 8, 20, 20)),       # fast res2 conv_a
    (8, 32, (1, 1, 1), (1, 1, 1), (0, 0, 0), (2, 8, 20, 20)),       # fast res2 conv_c / branch1
    (16, 16, (1, 3, 3), (1, 2, 2), (0, 1, 1), (2, 8, 28, 28)),      # fast res3 conv_b, stride 2
    (16, 64, (1, 1, 1), (1, 1, 1), (0, 0, 0), (2, 8, 14, 14)),      # fast res3 conv_c (N = 64)
    (64, 48, (3, 1, 1), (1, 1, 1), (1, 0, 0), (2, 8, 14, 14)),      # NB = 3, K = 192
    (8, 16, (7, 1, 1), (4, 1, 1), (3, 0, 0), (2, 32, 14, 14)),      # lateral fusion fuse0
    (32, 64, (1, 1, 1), (1, 2, 2), (0, 0, 0), (2, 8, 14, 14)),      # fast branch1 stride 2
    (64, 64, (1, 3, 3), (1, 1, 1), (0, 1, 1), (2, 4, 7, 7)),        # fast res5 conv_b, K = 576
]
CFGS = [EXPLICIT | DIRECT, EXPLICIT | DIRECT | DIRECT_2K, EXPLICIT | DIRECT | DIRECT_HALF,
        EXPLICIT | DIRECT | DIRECT_2K | DIRECT_HALF]


def C():
    from pytorchvideo_accelerate_amd.ops._ext import require
    return require()


def rel_err(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6)).item()


def _mk(case, seed):
    cin, cout, k, s, p, (N, T, H, W) = case
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(N, cin, T, H, W, generator=g).to(DEV).to(torch.bfloat16).float()
    w = (torch.randn(cout, cin, *k, generator=g) / (cin * k[0] * k[1] * k[2]) ** 0.5).to(DEV)
    return x, w.to(torch.bfloat16).float(), ConvSpec(cin, cout, k, s, p)


@pytest.mark.parametrize("cfg", CFGS)
@pytest.mark.parametrize("case", CASES)
def test_direct_fwd_affine_stats(case, cfg):
    x, w, spec = _mk(case, 31)
    Cin = spec.cin
    sc = torch.rand(Cin, device=DEV) + 0.5
    sh = torch.randn(Cin, device=DEV) * 0.5
    xa = Act.from_ncthw(x)
    xt = torch.relu(x * sc.view(1, Cin, 1, 1, 1) + sh.view(1, Cin, 1, 1, 1))
    ref = torch.nn.functional.conv3d(xt, w, None, spec.stride, spec.pad)
    wf, _ = pack_weight(w, spec)
    To, Ho, Wo = spec.out_dims(xa.T, xa.H, xa.W)
    M = xa.N * To * Ho * Wo
    g = fwd_geometry(spec, xa.N, xa.T, xa.H, xa.W, xa.ld, spec.cout)
    assert C().conv_direct_legal(g, 8) == 1
    rows = C().conv_cfg_bm(cfg, spec.cout)
    stats = torch.full(((M + rows - 1) // rows, 2, spec.cout), float("nan"), device=DEV)
    y = torch.empty(M, spec.cout, device=DEV, dtype=torch.bfloat16)
    C().conv_igemm(xa.t, wf, y, stats, sc, sh, 2, 0, g, 8, cfg)
    assert rel_err(Act(y, xa.N, To, Ho, Wo).to_ncthw(), ref) < 1.5e-2
    yf = y.float()
    torch.testing.assert_close(stats.sum(0)[0], yf.sum(0), rtol=1e-3,
                               atol=1e-2 * yf.abs().sum(0).max().item() / M ** 0.5)
    torch.testing.assert_close(stats.sum(0)[1], (yf * yf).sum(0), rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("cfg", CFGS[::2])
@pytest.mark.parametrize("case", CASES)
def test_direct_dgrad_phases_accum(case, cfg):
    x, w, spec = _mk(case, 32)
    if spec.cin > 64:
        pytest.skip("dgrad N = Cin > 64")
    N, Ci, T, H, W = x.shape
    ref_y = torch.nn.functional.conv3d(x, w, None, spec.stride, spec.pad)
    gy = torch.randn_like(ref_y).to(torch.bfloat16).float()
    dx_ref = torch.nn.grad.conv3d_input(x.shape, w, gy, spec.stride, spec.pad)
    _, wd = pack_weight(w, spec)
    dy = Act.from_ncthw(gy)
    M = N * T * H * W
    out = torch.zeros(M, Ci, device=DEV, dtype=torch.bfloat16)
    for g in dgrad_phases(spec, N, (T, H, W), (dy.T, dy.H, dy.W), dy.ld, Ci):
        if g[28] == 0:
            continue  # phase without contributing taps: zeros already there
        assert C().conv_direct_legal(g, 8) == 1
        C().conv_igemm(dy.t, wd, out, None, None, None, 0, 0, g, 8, cfg)
    dxa = Act(out, N, T, H, W)
    assert rel_err(dxa.to_ncthw(), dx_ref) < 1e-2
    out2 = out.clone()
    for g in dgrad_phases(spec, N, (T, H, W), (dy.T, dy.H, dy.W), dy.ld, Ci):
        if g[28]:
            C().conv_igemm(dy.t, wd, out2, None, None, None, 0, 1, g, 8, cfg)
    assert rel_err(Act(out2, N, T, H, W).to_ncthw(), 2 * dx_ref) < 1.5e-2


def _bits(mask):
    M, Ch = mask.shape
    w = (1 << torch.arange(8, device=mask.device)).to(torch.int32)
    return (mask.view(M, Ch // 8, 8).to(torch.int32) * w).sum(-1).to(torch.uint8)


@pytest.mark.parametrize("cfg", CFGS[::2])
@pytest.mark.parametrize("mode", ["dual_accum", "single", "affine_mask"])
@pytest.mark.parametrize("case", [CASES[1], CASES[4], (64, 32, (3, 1, 1), (1, 1, 1), (1, 0, 0), (2, 8, 14, 14))])
def test_direct_dgrad_bn_epilogue(case, mode, cfg):
    x, w, spec = _mk(case, 33)
    N, Ci, T, H, W = x.shape
    if Ci > 64 or Ci % 8:
        pytest.skip("dgrad N = Cin must be <= 64 and a multiple of 8")
    ref_y = torch.nn.functional.conv3d(x, w, None, spec.stride, spec.pad)
    gy = torch.randn_like(ref_y).to(torch.bfloat16).float()
    dx_ref = torch.nn.grad.conv3d_input(x.shape, w, gy, spec.stride, spec.pad).permute(0, 2, 3, 4, 1)
    M = N * T * H * W
    dx_ref = dx_ref.reshape(M, Ci)
    gen = torch.Generator(device="cpu").manual_seed(34)
    bf = lambda *s: torch.randn(*s, generator=gen).to(torch.bfloat16).to(DEV)
    res, old, y0, y1 = bf(M, Ci), bf(M, Ci), bf(M, Ci) * 2 + 0.5, bf(M, Ci)
    mask = torch.rand(M, Ci, generator=gen).to(DEV) > 0.4
    mean0, rstd0 = torch.randn(Ci, device=DEV) * 0.3, torch.rand(Ci, device=DEV) + 0.5
    mean1, rstd1 = torch.randn(Ci, device=DEV) * 0.3, torch.rand(Ci, device=DEV) + 0.5
    msc, msh = torch.rand(Ci, device=DEV) + 0.2, torch.randn(Ci, device=DEV) * 0.5
    _, wd = pack_weight(w, spec)
    dy = Act.from_ncthw(gy)
    geo = dgrad_phases(spec, N, (T, H, W), (dy.T, dy.H, dy.W), dy.ld, Ci)
    assert len(geo) == 1
    rows = C().conv_cfg_bm(cfg, Ci)
    part = torch.full(((M + rows - 1) // rows, 3, Ci), float("nan"), device=DEV)
    if mode == "dual_accum":
        out = old.clone()
        C().conv_igemm_epi(dy.t, wd, out, 1, geo[0], 8, res, Ci, _bits(mask), y0, mean0, rstd0, y1, mean1, rstd1,
                           part, None, None, cfg)
        v = (dx_ref + old.float() + res.float()) * mask
    elif mode == "single":
        out = torch.empty_like(old)
        C().conv_igemm_epi(dy.t, wd, out, 0, geo[0], 8, None, 0, _bits(mask), y0, mean0, rstd0, None, None, None,
                           part, None, None, cfg)
        v = dx_ref * mask
    else:
        out = torch.empty_like(old)
        C().conv_igemm_epi(dy.t, wd, out, 0, geo[0], 8, None, 0, None, y0, mean0, rstd0, None, None, None,
                           part, msc, msh, cfg)
        v = dx_ref * ((y0.float() * msc + msh) > 0)
    assert rel_err(out, v) < 1.5e-2
    q = out.float()
    s = part.sum(0)
    tol = 2e-2 * (q.abs() * (y0.float() - mean0).abs() * rstd0).sum(0).max().item() / M ** 0.5
    torch.testing.assert_close(s[0], q.sum(0), rtol=1e-3, atol=1e-2 * q.abs().sum(0).max().item() / M ** 0.5)
    torch.testing.assert_close(s[1], (q * (y0.float() - mean0) * rstd0).sum(0), rtol=1e-3, atol=tol)
    if mode == "dual_accum":
        torch.testing.assert_close(s[2], (q * (y1.float() - mean1) * rstd1).sum(0), rtol=1e-3, atol=tol)
