"""Halo-staged (1,3,3) conv kernels (csrc/kernels/conv_halo.hip, wide and narrow) and the box-staged weight
gradient (csrc/kernels/wgrad_box.hip) against plain PyTorch fp32 references:
forward with the consumer-side BN+ReLU prologue and the BN partial sums, eval forward, plain dgrad, and the
dgrad epilogue of a conv whose input is relu(BN_a(y0)) (ReLU mask from y0 + BN_a backward partials) — at the
slow-pathway conv_b shapes (64/128/256 channels at 56/28/14 px; R101's 64 px), both n-tile widths, and the fast
pathway's 8/16/32-channel conv_b (narrow variant)."""
import pytest
import torch
import torch.nn.functional as F

from pytorchvideo_accelerate_amd.ops._ext import require
from pytorchvideo_accelerate_amd.ops.conv import Act, ConvSpec, conv_dgrad, conv_fwd, dgrad_phases, fwd_geometry, pack_weight

pytestmark = pytest.mark.gpu
DEV = "cuda"
HALO, EXPLICIT = 2048, 16

# (channels, N, T, H, W)
CASES = [
    (64, 1, 2, 56, 56),     # slow res2 conv_b (224-position tiles)
    (128, 1, 3, 28, 28),    # slow res3 conv_b (196-position tiles, partial MFMA block)
    (256, 2, 2, 14, 14),    # slow res4 conv_b (two 128-channel halo slices)
    (64, 1, 1, 64, 64),     # R101 256-crop res2 (128-position tiles)
    (64, 4, 8, 56, 56),     # 448 tiles: several tiles per workgroup of the persistent 64-channel variant
    (8, 2, 3, 56, 56),      # fast res2 conv_b (narrow variant, 784-position tiles)
    (16, 1, 4, 28, 28),     # fast res3 conv_b (narrow, whole frames)
    (32, 2, 2, 14, 14),     # fast res4 conv_b (narrow, 196-position tiles)
]


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6)).item()


def _mk(C, N, T, H, W, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, C, T, H, W, generator=g).to(torch.bfloat16).float().to(DEV)
    w = (torch.randn(C, C, 1, 3, 3, generator=g) / (9 * C) ** 0.5).to(torch.bfloat16).float().to(DEV)
    return x, w, ConvSpec(C, C, (1, 3, 3), (1, 1, 1), (0, 1, 1))


def _cfgs(g, C):
    P = require().conv_halo_legal(list(g), 8)
    assert P > 0, "halo kernel must accept this geometry"
    base = EXPLICIT | HALO | (P << 12)
    cfgs = [base, base | 1] if C % 128 == 0 else [base | 1]
    lg = require().conv_halo64p_legal(list(g), 8)
    if lg:   # persistent 64-channel variant, 256 / 1024 workgroups
        cfgs += [base | 1 | 2, base | 1 | 2 | 4]
    if lg == 2:   # double-buffered 8x28-tile variant
        cfgs += [base | 1 | 2 | 8, base | 1 | 2 | 8 | 4]
    return P, cfgs


@pytest.mark.parametrize("case", CASES)
def test_halo_forward_affine_stats(case):
    C, N, T, H, W = case
    x, w, spec = _mk(C, N, T, H, W, seed=3)
    sc = (torch.rand(C, device=DEV) + 0.5)
    sh = torch.randn(C, device=DEV) * 0.5
    xt = torch.relu(x * sc.view(1, C, 1, 1, 1) + sh.view(1, C, 1, 1, 1)).to(torch.bfloat16).float()
    ref = F.conv3d(xt, w, None, spec.stride, spec.pad)
    wf, _ = pack_weight(w, spec)
    xa = Act.from_ncthw(x)
    g = fwd_geometry(spec, N, T, H, W, xa.ld, C)
    P, cfgs = _cfgs(g, C)
    M = N * T * H * W
    for cfg in cfgs:
        stats = torch.full((M // P, 2, C), float("nan"), device=DEV)
        y = conv_fwd(xa, wf, spec, stats=stats, in_scale=sc, in_shift=sh, in_relu=True, cfg=cfg)
        assert _rel(y.to_ncthw(), ref) < 1e-2, cfg
        yf = y.t.float()
        s = stats.sum(0)
        torch.testing.assert_close(s[0], yf.sum(0), rtol=1e-4, atol=1e-3 * yf.abs().sum(0).max().item() / M ** 0.5)
        torch.testing.assert_close(s[1], (yf * yf).sum(0), rtol=1e-4, atol=1e-3)
        # eval form: no affine, no statistics
        ye = conv_fwd(xa, wf, spec, cfg=cfg)
        assert _rel(ye.to_ncthw(), F.conv3d(x, w, None, spec.stride, spec.pad)) < 1e-2


@pytest.mark.parametrize("case", CASES)
def test_halo_dgrad_and_bn_epilogue(case):
    C, N, T, H, W = case
    x, w, spec = _mk(C, N, T, H, W, seed=4)
    gy = torch.randn(N, C, T, H, W, generator=torch.Generator().manual_seed(5)).to(torch.bfloat16).float().to(DEV)
    dx_ref = torch.nn.grad.conv3d_input(x.shape, w, gy, spec.stride, spec.pad)
    _, wd = pack_weight(w, spec)
    dy = Act.from_ncthw(gy)
    geo = dgrad_phases(spec, N, (T, H, W), (T, H, W), dy.ld, C)
    assert len(geo) == 1
    P, cfgs = _cfgs(geo[0], C)
    Cm = require()
    M = N * T * H * W
    # y0: the raw conv output feeding this conv through relu(BN(y0)); mask and BN_a partials
    y0 = torch.randn(M, C, generator=torch.Generator().manual_seed(6)).to(torch.bfloat16).to(DEV)
    mean0 = torch.randn(C, device=DEV) * 0.1
    rstd0 = torch.rand(C, device=DEV) + 0.5
    msc = torch.rand(C, device=DEV) + 0.5
    msh = torch.randn(C, device=DEV) * 0.3
    y0f = y0.float()
    mask = (y0f * msc + msh > 0).float()
    for cfg in cfgs:
        dx = conv_dgrad(dy, wd, spec, (T, H, W), cfg=cfg)
        assert _rel(dx.to_ncthw(), dx_ref) < 1e-2, cfg
        out = torch.empty(M, C, device=DEV, dtype=torch.bfloat16)
        part = torch.full((M // P, 3, C), float("nan"), device=DEV)
        Cm.conv_igemm_epi(dy.t, wd, out, 0, geo[0], 8, None, 0, None, y0, mean0, rstd0, None, None, None, part,
                          msc, msh, cfg, None)
        v_ref = Act.from_ncthw(dx_ref).t.float() * mask
        assert _rel(out.float(), v_ref) < 1e-2
        q = out.float()
        ps = part.sum(0)
        torch.testing.assert_close(ps[0], q.sum(0), rtol=1e-3, atol=1e-3 * q.abs().sum(0).max().item() / M ** 0.5)
        xhat = (y0f - mean0) * rstd0
        torch.testing.assert_close(ps[1], (q * xhat).sum(0), rtol=1e-3,
                                   atol=1e-3 * (q * xhat).abs().sum(0).max().item() / M ** 0.5)
        assert torch.all(ps[2] == 0)


def test_halo_legality():
    """Geometries the halo kernel must refuse: strided, temporal taps, too-narrow tiles, odd channel counts."""
    Cm = require()
    ok = fwd_geometry(ConvSpec(64, 64, (1, 3, 3), (1, 1, 1), (0, 1, 1)), 2, 4, 56, 56, 64, 64)
    assert Cm.conv_halo_legal(ok, 8) == 224
    assert Cm.conv_halo_legal(fwd_geometry(ConvSpec(64, 64, (1, 3, 3), (1, 2, 2), (0, 1, 1)), 2, 4, 56, 56, 64, 64), 8) == 0
    assert Cm.conv_halo_legal(fwd_geometry(ConvSpec(64, 64, (3, 1, 1), (1, 1, 1), (1, 0, 0)), 2, 4, 56, 56, 64, 64), 8) == 0
    assert Cm.conv_halo_legal(fwd_geometry(ConvSpec(512, 512, (1, 3, 3), (1, 1, 1), (0, 1, 1)), 2, 4, 7, 7, 512, 512), 8) == 0
    assert Cm.conv_halo_legal(fwd_geometry(ConvSpec(24, 24, (1, 3, 3), (1, 1, 1), (0, 1, 1)), 2, 4, 56, 56, 24, 24), 8) == 0
    assert Cm.conv_halo_legal(fwd_geometry(ConvSpec(16, 16, (1, 3, 3), (1, 1, 1), (0, 1, 1)), 2, 4, 56, 56, 16, 16), 8) == 784
    assert Cm.conv_halo64p_legal(ok, 8) == 2   # persistent and double-buffered variants
    assert Cm.conv_halo64p_legal(fwd_geometry(ConvSpec(64, 64, (1, 3, 3), (1, 1, 1), (0, 1, 1)), 1, 1, 64, 64, 64, 64), 8) == 1
    assert Cm.conv_halo64p_legal(fwd_geometry(ConvSpec(128, 128, (1, 3, 3), (1, 1, 1), (0, 1, 1)), 2, 4, 28, 28, 128, 128), 8) == 0


WGRAD_CASES = [(64, 1, 2, 56, 56), (128, 1, 3, 28, 28), (256, 2, 2, 14, 14), (64, 1, 1, 64, 64),
               (8, 2, 3, 56, 56), (16, 1, 4, 28, 28), (32, 2, 2, 14, 14)]


@pytest.mark.parametrize("case", WGRAD_CASES)
def test_box_wgrad_vs_torch(case):
    """Box-staged weight gradient (csrc/kernels/wgrad_box.hip) with the producer's BN+ReLU recomputed on the input
    halo, against torch.nn.grad.conv3d_weight in fp32; accumulate (beta) and scale through the slab reduction."""
    from pytorchvideo_accelerate_amd.ops.conv import BOX, box_wgrad_plan, conv_wgrad
    C, N, T, H, W = case
    x, w, spec = _mk(C, N, T, H, W, seed=7)
    sc = torch.rand(C, device=DEV) + 0.5
    sh = torch.randn(C, device=DEV) * 0.5
    xt = torch.relu(x * sc.view(1, C, 1, 1, 1) + sh.view(1, C, 1, 1, 1)).to(torch.bfloat16).float()
    gy = torch.randn(N, C, T, H, W, generator=torch.Generator().manual_seed(8)).to(torch.bfloat16).float().to(DEV)
    ref = torch.nn.grad.conv3d_weight(xt, w.shape, gy, spec.stride, spec.pad)
    xa, dy = Act.from_ncthw(x), Act.from_ncthw(gy)
    assert box_wgrad_plan(spec, dy.M, (T, H, W), dy.ld, xa.ld) is not None
    grad = torch.full_like(ref, float("nan"))
    conv_wgrad(dy, xa, spec, grad, in_scale=sc, in_shift=sh, in_relu=True, variant=BOX)
    assert _rel(grad, ref) < 5e-3
    prev = grad.clone()
    conv_wgrad(dy, xa, spec, grad, in_scale=sc, in_shift=sh, in_relu=True, variant=BOX, scale=0.5, beta=1.0)
    assert _rel(grad, prev + 0.5 * ref) < 5e-3
    # bitwise reproducible (fixed-order slab reduction, no atomics)
    g2 = torch.empty_like(ref)
    conv_wgrad(dy, xa, spec, g2, in_scale=sc, in_shift=sh, in_relu=True, variant=BOX)
    assert torch.equal(g2, prev)
