"""Numerics of the gfx950 HIP kernels against plain PyTorch fp32 references of the same op.

Random (non-zero) data, every conv class of SlowFast-R50 at a reduced batch:
pointwise / temporal / spatial / stride-2 / lateral fusion / both stems / tiny-channel fast pathway.
"""
import pytest
import torch

from pytorchvideo_accelerate_amd.ops.conv import Act, ConvSpec, conv_dgrad, conv_fwd, conv_wgrad, pack_weight

pytestmark = pytest.mark.gpu

DEV = "cuda"

# (cin, cout, k, stride, pad, (N, T, H, W))
CASES = [
    (64, 256, (1, 1, 1), (1, 1, 1), (0, 0, 0), (2, 4, 14, 14)),      # slow pointwise
    (256, 64, (3, 1, 1), (1, 1, 1), (1, 0, 0), (2, 8, 14, 14)),      # slow temporal
    (64, 64, (1, 3, 3), (1, 1, 1), (0, 1, 1), (2, 4, 14, 14)),       # slow spatial
    (128, 128, (1, 3, 3), (1, 2, 2), (0, 1, 1), (2, 4, 28, 28)),     # spatial stride 2
    (320, 512, (1, 1, 1), (1, 2, 2), (0, 0, 0), (2, 4, 14, 14)),     # branch1 stride 2
    (8, 16, (7, 1, 1), (4, 1, 1), (3, 0, 0), (2, 32, 14, 14)),       # lateral fusion
    (8, 8, (3, 1, 1), (1, 1, 1), (1, 0, 0), (2, 16, 14, 14)),        # fast temporal, N=8
    (16, 16, (1, 3, 3), (1, 2, 2), (0, 1, 1), (2, 8, 14, 14)),       # fast spatial s2
    (32, 8, (3, 1, 1), (1, 1, 1), (1, 0, 0), (2, 16, 7, 7)),         # fast conv_a
    (80, 64, (1, 1, 1), (1, 1, 1), (0, 0, 0), (2, 4, 14, 14)),       # concat input (80 ch)
    (512, 2048, (1, 1, 1), (1, 1, 1), (0, 0, 0), (2, 2, 7, 7)),      # res5 conv_c
]

STEMS = [
    (3, 64, (1, 7, 7), (1, 2, 2), (0, 3, 3), (2, 2, 32, 32)),
    (3, 8, (5, 7, 7), (1, 2, 2), (2, 3, 3), (2, 6, 32, 32)),
]


def rel_err(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6)).item()


def _mk(case, seed=0):
    cin, cout, k, s, p, (N, T, H, W) = case
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(N, cin, T, H, W, generator=g).to(DEV).to(torch.bfloat16).float()
    w = (torch.randn(cout, cin, *k, generator=g) / (cin * k[0] * k[1] * k[2]) ** 0.5).to(DEV)
    w = w.to(torch.bfloat16).float()
    spec = ConvSpec(cin, cout, k, s, p, cin_pad=4 if cin == 3 else 0)
    return x, w, spec


@pytest.mark.parametrize("case", CASES + STEMS)
def test_conv_fwd(case):
    x, w, spec = _mk(case)
    ref = torch.nn.functional.conv3d(x, w, None, spec.stride, spec.pad)
    wf, _ = pack_weight(w, spec)
    xa = Act.from_ncthw(x, spec.cin_pad)
    y = conv_fwd(xa, wf, spec)
    assert rel_err(y.to_ncthw(), ref) < 1e-2


@pytest.mark.parametrize("case", CASES[:4])
def test_conv_fwd_stats_and_affine(case):
    x, w, spec = _mk(case, seed=1)
    C = spec.cin
    sc = torch.rand(C, device=DEV) + 0.5
    sh = torch.randn(C, device=DEV) * 0.5
    xa = Act.from_ncthw(x)
    xt = torch.relu(x * sc.view(1, C, 1, 1, 1) + sh.view(1, C, 1, 1, 1))
    ref = torch.nn.functional.conv3d(xt, w, None, spec.stride, spec.pad)
    wf, _ = pack_weight(w, spec)
    from pytorchvideo_accelerate_amd.ops.conv import conv_m_tiles
    To, Ho, Wo = spec.out_dims(xa.T, xa.H, xa.W)
    M = xa.N * To * Ho * Wo
    tiles = conv_m_tiles(M, spec.cout, spec)
    stats = torch.empty(tiles, 2, spec.cout, device=DEV)
    y = conv_fwd(xa, wf, spec, stats=stats, in_scale=sc, in_shift=sh, in_relu=True)
    assert rel_err(y.to_ncthw(), ref) < 1.5e-2
    yf = y.t.float()
    s = stats.sum(0)
    torch.testing.assert_close(s[0], yf.sum(0), rtol=1e-3, atol=1e-2 * yf.abs().sum(0).max().item() / M ** 0.5)
    torch.testing.assert_close(s[1], (yf * yf).sum(0), rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("case", [c for c in CASES if c[0] % 8 == 0])
def test_conv_dgrad(case):
    x, w, spec = _mk(case, seed=2)
    x.requires_grad_(True)
    ref_y = torch.nn.functional.conv3d(x, w, None, spec.stride, spec.pad)
    gy = torch.randn_like(ref_y).to(torch.bfloat16).float()
    ref_y.backward(gy)
    _, wd = pack_weight(w, spec)
    dy = Act.from_ncthw(gy)
    dx = conv_dgrad(dy, wd, spec, tuple(x.shape[2:]))
    assert rel_err(dx.to_ncthw(), x.grad) < 1e-2
    # accumulate mode
    dx2 = conv_dgrad(dy, wd, spec, tuple(x.shape[2:]), out=dx.t.clone(), accum=True)
    assert rel_err(dx2.to_ncthw(), 2 * x.grad) < 1.5e-2


# fast-pathway shapes at realistic row counts (M >= 32768): small-channel tiles, strided dgrad phases
STREAM_CASES = [
    (8, 8, (1, 3, 3), (1, 1, 1), (0, 1, 1), (2, 16, 40, 40)),      # fast res2 conv_b
    (32, 8, (3, 1, 1), (1, 1, 1), (1, 0, 0), (2, 16, 32, 32)),     # fast res2 conv_a
    (8, 32, (1, 1, 1), (1, 1, 1), (0, 0, 0), (2, 16, 32, 32)),     # fast res2 conv_c
    (16, 16, (1, 3, 3), (1, 2, 2), (0, 1, 1), (2, 16, 64, 64)),    # fast res3 conv_b stride 2
    (16, 64, (1, 1, 1), (1, 1, 1), (0, 0, 0), (2, 16, 32, 32)),    # fast res3 conv_c (N = 64)
    (64, 16, (3, 1, 1), (1, 1, 1), (1, 0, 0), (2, 16, 32, 32)),    # K = 192 (KC = 32 variant)
]


@pytest.mark.parametrize("case", STREAM_CASES)
def test_small_channel_fwd_stats_affine_dgrad(case):
    from pytorchvideo_accelerate_amd.ops._ext import require
    from pytorchvideo_accelerate_amd.ops.conv import conv_m_tiles
    C = require()
    x, w, spec = _mk(case, seed=21)
    Cin = spec.cin
    sc = torch.rand(Cin, device=DEV) + 0.5
    sh = torch.randn(Cin, device=DEV) * 0.5
    xa = Act.from_ncthw(x)
    xt = torch.relu(x * sc.view(1, Cin, 1, 1, 1) + sh.view(1, Cin, 1, 1, 1))
    ref = torch.nn.functional.conv3d(xt, w, None, spec.stride, spec.pad)
    wf, wd = pack_weight(w, spec)
    To, Ho, Wo = spec.out_dims(xa.T, xa.H, xa.W)
    M = xa.N * To * Ho * Wo
    assert M >= 32768
    stats = torch.full((conv_m_tiles(M, spec.cout, spec), 2, spec.cout), float("nan"), device=DEV)
    y = conv_fwd(xa, wf, spec, stats=stats, in_scale=sc, in_shift=sh, in_relu=True)
    assert rel_err(y.to_ncthw(), ref) < 1.5e-2
    yf = y.t.float()
    torch.testing.assert_close(stats.sum(0)[0], yf.sum(0), rtol=1e-3, atol=1e-2 * yf.abs().sum(0).max().item() / M ** 0.5)
    torch.testing.assert_close(stats.sum(0)[1], (yf * yf).sum(0), rtol=1e-3, atol=1e-3)
    # dgrad (incl. stride-2 phases) and accumulate through the same kernel family
    gy = torch.randn_like(ref).to(torch.bfloat16).float()
    dx_ref = torch.nn.grad.conv3d_input(x.shape, w, gy, spec.stride, spec.pad)
    dy = Act.from_ncthw(gy)
    dx = conv_dgrad(dy, wd, spec, tuple(x.shape[2:]))
    assert rel_err(dx.to_ncthw(), dx_ref) < 1e-2
    dx2 = conv_dgrad(dy, wd, spec, tuple(x.shape[2:]), out=dx.t.clone(), accum=True)
    assert rel_err(dx2.to_ncthw(), 2 * dx_ref) < 1.5e-2


def _bits(mask):
    """bool [M, C] -> uint8 [M, C/8] with bit e of byte j = mask[:, 8j+e] (res_out's layout)."""
    M, C = mask.shape
    w = (1 << torch.arange(8, device=mask.device)).to(torch.int32)
    return (mask.view(M, C // 8, 8).to(torch.int32) * w).sum(-1).to(torch.uint8)


@pytest.mark.parametrize("case,dual,accum", [(CASES[1], True, False), (CASES[0], False, True),
                                             (CASES[8], True, True)])
def test_conv_dgrad_bn_epilogue(case, dual, accum):
    """dgrad + residual + ReLU-bit mask + backward-BN partial sums (sum v, sum v*xhat0, sum v*xhat1)."""
    from pytorchvideo_accelerate_amd.ops._ext import require
    from pytorchvideo_accelerate_amd.ops.conv import conv_m_tiles, dgrad_phases
    C = require()
    x, w, spec = _mk(case, seed=5)
    N, Ci, T, H, W = x.shape
    ref_y = torch.nn.functional.conv3d(x, w, None, spec.stride, spec.pad)
    gy = torch.randn_like(ref_y).to(torch.bfloat16).float()
    dx_ref = torch.nn.grad.conv3d_input(x.shape, w, gy, spec.stride, spec.pad)
    M = N * T * H * W
    g = torch.Generator(device="cpu").manual_seed(6)
    bf = lambda *s: torch.randn(*s, generator=g).to(torch.bfloat16).to(DEV)
    res, old, y0, y1 = bf(M, Ci), bf(M, Ci), bf(M, Ci) * 2 + 0.5, bf(M, Ci)
    mask = torch.rand(M, Ci, generator=g).to(DEV) > 0.4
    mean0, rstd0 = torch.randn(Ci, device=DEV) * 0.3, torch.rand(Ci, device=DEV) + 0.5
    mean1, rstd1 = torch.randn(Ci, device=DEV) * 0.3, torch.rand(Ci, device=DEV) + 0.5
    _, wd = pack_weight(w, spec)
    dy = Act.from_ncthw(gy)
    out = old.clone()
    geo = dgrad_phases(spec, N, (T, H, W), (dy.T, dy.H, dy.W), dy.ld, Ci)
    assert len(geo) == 1
    tiles = conv_m_tiles(M, Ci)
    part = torch.full((tiles, 3, Ci), float("nan"), device=DEV)
    C.conv_igemm_epi(dy.t, wd, out, 1 if accum else 0, geo[0], 8, res, Ci, _bits(mask), y0, mean0, rstd0,
                     y1 if dual else None, mean1 if dual else None, rstd1 if dual else None, part)
    dxr = dx_ref.permute(0, 2, 3, 4, 1).reshape(M, Ci)
    v = (dxr + (old.float() if accum else 0) + res.float()) * mask
    assert rel_err(out, v) < 1.5e-2
    q = out.float()
    s = part.sum(0)
    tol = 2e-2 * (q.abs() * (y0.float() - mean0).abs() * rstd0).sum(0).max().item() / M ** 0.5
    torch.testing.assert_close(s[0], q.sum(0), rtol=1e-3, atol=1e-2 * q.abs().sum(0).max().item() / M ** 0.5)
    torch.testing.assert_close(s[1], (q * (y0.float() - mean0) * rstd0).sum(0), rtol=1e-3, atol=tol)
    if dual:
        torch.testing.assert_close(s[2], (q * (y1.float() - mean1) * rstd1).sum(0), rtol=1e-3, atol=tol)


@pytest.mark.parametrize("case", [CASES[0], CASES[2], CASES[6]])
def test_conv_dgrad_bn_epilogue_affine_mask(case):
    """dgrad epilogue for a conv whose input is relu(BN(y)): v *= (y*scale + shift > 0) + BN partial sums."""
    from pytorchvideo_accelerate_amd.ops._ext import require
    from pytorchvideo_accelerate_amd.ops.conv import conv_m_tiles, dgrad_phases
    C = require()
    x, w, spec = _mk(case, seed=11)
    N, Ci, T, H, W = x.shape
    ref_y = torch.nn.functional.conv3d(x, w, None, spec.stride, spec.pad)
    gy = torch.randn_like(ref_y).to(torch.bfloat16).float()
    dx_ref = torch.nn.grad.conv3d_input(x.shape, w, gy, spec.stride, spec.pad)
    M = N * T * H * W
    g = torch.Generator(device="cpu").manual_seed(12)
    y0 = (torch.randn(M, Ci, generator=g) * 2 + 0.3).to(torch.bfloat16).to(DEV)
    mean0, rstd0 = torch.randn(Ci, device=DEV) * 0.3, torch.rand(Ci, device=DEV) + 0.5
    msc, msh = torch.rand(Ci, device=DEV) + 0.2, torch.randn(Ci, device=DEV) * 0.5
    _, wd = pack_weight(w, spec)
    dy = Act.from_ncthw(gy)
    out = torch.empty(M, Ci, device=DEV, dtype=torch.bfloat16)
    geo = dgrad_phases(spec, N, (T, H, W), (dy.T, dy.H, dy.W), dy.ld, Ci)
    part = torch.full((conv_m_tiles(M, Ci), 3, Ci), float("nan"), device=DEV)
    C.conv_igemm_epi(dy.t, wd, out, 0, geo[0], 8, None, 0, None, y0, mean0, rstd0, None, None, None, part,
                     msc, msh)
    mask = (y0.float() * msc + msh) > 0
    v = dx_ref.permute(0, 2, 3, 4, 1).reshape(M, Ci) * mask
    assert rel_err(out, v) < 1.5e-2
    q = out.float()
    s = part.sum(0)
    tol = 2e-2 * (q.abs() * (y0.float() - mean0).abs() * rstd0).sum(0).max().item() / M ** 0.5
    torch.testing.assert_close(s[0], q.sum(0), rtol=1e-3, atol=1e-2 * q.abs().sum(0).max().item() / M ** 0.5)
    torch.testing.assert_close(s[1], (q * (y0.float() - mean0) * rstd0).sum(0), rtol=1e-3, atol=tol)


def test_res_out_mask_bits():
    from pytorchvideo_accelerate_amd.ops._ext import require
    C = require()
    M, Ch = 1000, 64
    g = torch.Generator(device="cpu").manual_seed(7)
    yc = torch.randn(M, Ch, generator=g).to(torch.bfloat16).to(DEV)
    x = torch.randn(M, Ch, generator=g).to(torch.bfloat16).to(DEV)
    sc, sh = torch.rand(Ch, device=DEV) + 0.5, torch.randn(Ch, device=DEV) * 0.1
    out = torch.empty(M, Ch, device=DEV, dtype=torch.bfloat16)
    mask = torch.zeros(M, Ch // 8, device=DEV, dtype=torch.uint8)
    C.res_out(yc, sc, sh, None, None, None, x, Ch, out, Ch, M, Ch, mask)
    ref = torch.relu(yc.float() * sc + sh + x.float())
    assert rel_err(out, ref) < 1e-2
    assert torch.equal(mask, _bits(out.float() > 0))


@pytest.mark.parametrize("case", CASES + STEMS)
def test_conv_wgrad(case):
    x, w, spec = _mk(case, seed=3)
    w.requires_grad_(True)
    ref_y = torch.nn.functional.conv3d(x, w, None, spec.stride, spec.pad)
    gy = torch.randn_like(ref_y).to(torch.bfloat16).float()
    ref_y.backward(gy)
    grad = torch.zeros_like(w)
    conv_wgrad(Act.from_ncthw(gy), Act.from_ncthw(x, spec.cin_pad), spec, grad)
    assert rel_err(grad, w.grad) < 1e-2
    # beta / scale accumulate
    conv_wgrad(Act.from_ncthw(gy), Act.from_ncthw(x, spec.cin_pad), spec, grad, scale=0.5, beta=1.0)
    assert rel_err(grad, 1.5 * w.grad) < 1e-2


@pytest.mark.parametrize("splits", [3, 8, 40, 300])
@pytest.mark.parametrize("case", [CASES[1], CASES[6], STEMS[1]])
def test_conv_wgrad_slab_reduction(case, splits):
    """Per-split slabs + the fixed-order slab reduction (every wave-count branch: 1, 4, 8, 16 waves per 64 entries;
    padded input channels skipped) against PyTorch, with beta/scale, and bitwise equal run to run."""
    x, w, spec = _mk(case, seed=5)
    w.requires_grad_(True)
    ref_y = torch.nn.functional.conv3d(x, w, None, spec.stride, spec.pad)
    gy = torch.randn_like(ref_y).to(torch.bfloat16).float()
    ref_y.backward(gy)
    dy, xa = Act.from_ncthw(gy), Act.from_ncthw(x, spec.cin_pad)
    pps = (dy.M + splits - 1) // splits
    pps = (pps + 31) // 32 * 32
    sp = ((dy.M + pps - 1) // pps, pps)
    grad = torch.zeros_like(w)
    conv_wgrad(dy, xa, spec, grad, splits_pps=sp, slab=True)
    assert rel_err(grad, w.grad) < 1e-2
    g2 = torch.full_like(w, 2.0)
    conv_wgrad(dy, xa, spec, g2, splits_pps=sp, slab=True, scale=0.5, beta=1.0)
    assert rel_err(g2, 2.0 + 0.5 * w.grad) < 1e-2
    again = torch.zeros_like(w)
    conv_wgrad(dy, xa, spec, again, splits_pps=sp, slab=True)
    assert torch.equal(grad, again)


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15])
@pytest.mark.parametrize("case", [CASES[1], CASES[3], CASES[6], STEMS[1]])
def test_conv_wgrad_tile_variants(case, variant):
    """Every tile variant (bits 0-1 + bit 3) x {32, 64}-position LDS stages (bit 2) against PyTorch."""
    x, w, spec = _mk(case, seed=13)
    w.requires_grad_(True)
    ref_y = torch.nn.functional.conv3d(x, w, None, spec.stride, spec.pad)
    gy = torch.randn_like(ref_y).to(torch.bfloat16).float()
    ref_y.backward(gy)
    grad = torch.zeros_like(w)
    conv_wgrad(Act.from_ncthw(gy), Act.from_ncthw(x, spec.cin_pad), spec, grad, variant=variant)
    assert rel_err(grad, w.grad) < 1e-2


@pytest.mark.parametrize("case", [CASES[5], CASES[6], CASES[8],
                                  (8, 8, (1, 3, 3), (1, 1, 1), (0, 1, 1), (2, 8, 15, 13)),
                                  (16, 16, (3, 1, 1), (1, 1, 1), (1, 0, 0), (3, 5, 7, 9)),
                                  (8, 16, (1, 1, 1), (1, 2, 2), (0, 0, 0), (2, 4, 14, 14)),
                                  (16, 32, (1, 1, 1), (1, 1, 1), (0, 0, 0), (2, 4, 9, 11)),
                                  (8, 24, (3, 1, 1), (1, 1, 1), (1, 0, 0), (2, 4, 7, 7)),
                                  (32, 32, (1, 1, 1), (1, 1, 1), (0, 0, 0), (2, 3, 10, 10))])
@pytest.mark.parametrize("affine", [False, True])
def test_conv_wgrad_narrow(case, affine):
    """Barrier-free per-wave wgrad kernel (Cout <= 32, K <= 128): padding, strides, odd sizes, BN-ReLU recompute."""
    x, w, spec = _mk(case, seed=21)
    C = spec.cin
    sc = torch.rand(C, device=DEV) + 0.5
    sh = torch.randn(C, device=DEV) * 0.5
    xt = torch.relu(x * sc.view(1, C, 1, 1, 1) + sh.view(1, C, 1, 1, 1)) if affine else x
    xt = xt.to(torch.bfloat16).float()
    w.requires_grad_(True)
    ref_y = torch.nn.functional.conv3d(xt, w, None, spec.stride, spec.pad)
    gy = torch.randn_like(ref_y).to(torch.bfloat16).float()
    ref_y.backward(gy)
    grad = torch.zeros_like(w)
    conv_wgrad(Act.from_ncthw(gy), Act.from_ncthw(x), spec, grad, in_scale=sc if affine else None,
               in_shift=sh if affine else None, variant=16)
    assert rel_err(grad, w.grad) < 1.5e-2


RT_CASES = [CASES[1], CASES[2], CASES[3], CASES[4], CASES[5], CASES[6], CASES[8],
            (64, 128, (3, 1, 1), (1, 1, 1), (1, 0, 0), (3, 5, 7, 9)),      # odd dims: positions past P
            (32, 64, (1, 3, 3), (1, 1, 1), (0, 1, 1), (2, 3, 5, 11))]


@pytest.mark.parametrize("tile", [2, 3, 4, 5, 6, 7])
@pytest.mark.parametrize("bp64", [False, True])
@pytest.mark.parametrize("affine", [False, True])
@pytest.mark.parametrize("case", RT_CASES)
def test_conv_wgrad_rowtable(case, tile, bp64, affine):
    """Row-table weight-gradient kernel (wgrad_rt_impl.h): every tile x stage depth, padding / strides / odd
    sizes, BN(+ReLU) recompute of X on load, and split-K with several (uneven) position splits."""
    from pytorchvideo_accelerate_amd.ops.conv import RT, wgrad_splits
    x, w, spec = _mk(case, seed=31)
    C = spec.cin
    sc = torch.rand(C, device=DEV) + 0.5
    sh = torch.randn(C, device=DEV) * 0.5
    xt = torch.relu(x * sc.view(1, C, 1, 1, 1) + sh.view(1, C, 1, 1, 1)) if affine else x
    xt = xt.to(torch.bfloat16).float()
    w.requires_grad_(True)
    ref_y = torch.nn.functional.conv3d(xt, w, None, spec.stride, spec.pad)
    gy = torch.randn_like(ref_y).to(torch.bfloat16).float()
    ref_y.backward(gy)
    dy = Act.from_ncthw(gy)
    v = (tile & 3) | (8 if tile >= 4 else 0)
    K = spec.taps * spec.cin_pad
    for tb in (64, 1024):   # one split, then many
        sp = wgrad_splits(dy.M, spec.cout, K, target_blocks=tb, min_rows=64, variant=v)
        grad = torch.zeros_like(w)
        conv_wgrad(dy, Act.from_ncthw(x), spec, grad, in_scale=sc if affine else None,
                   in_shift=sh if affine else None, splits_pps=sp, variant=RT | v | (4 if bp64 else 0))
        assert rel_err(grad, w.grad) < 1.5e-2, (tb, sp)


def test_conv_wgrad_affine():
    case = CASES[2]
    x, w, spec = _mk(case, seed=4)
    C = spec.cin
    sc = torch.rand(C, device=DEV) + 0.5
    sh = torch.randn(C, device=DEV) * 0.5
    xt = torch.relu(x * sc.view(1, C, 1, 1, 1) + sh.view(1, C, 1, 1, 1))
    w.requires_grad_(True)
    ref_y = torch.nn.functional.conv3d(xt, w, None, spec.stride, spec.pad)
    gy = torch.randn_like(ref_y).to(torch.bfloat16).float()
    ref_y.backward(gy)
    grad = torch.zeros_like(w)
    conv_wgrad(Act.from_ncthw(gy), Act.from_ncthw(x), spec, grad, in_scale=sc, in_shift=sh)
    assert rel_err(grad, w.grad) < 1.5e-2


def test_pack_weights_kernel_matches_host_pack():
    from pytorchvideo_accelerate_amd.models import reference as R
    from pytorchvideo_accelerate_amd.models.fused import FusedNet
    torch.manual_seed(0)
    eng = FusedNet(R.create_slowfast(50, 10), torch.device(DEV))
    for u in eng.units:
        wf, wd = pack_weight(u.conv.weight.detach(), u.spec)
        assert torch.equal(u.wf.view_as(wf), wf), u.name
        if u.wd is not None:
            assert torch.equal(u.wd.view_as(wd), wd), u.name


# (5, 8): frame-pair kernels (arm stem_pair, PVA_ARMS, default) for T = 4k .. 4k+3, and the one-frame kernels
# (1, 64): the slow stem with the channel-permuted 16-B-store epilogue (default) and without (stem_perm=0);
# roll "0": the frame-pair wgrad with one tap row per wave instead of the rolling-fragment default (stem_roll=0);
# roll "s": the rolling form with intrinsic (synchronous) transpose reads instead of the asm ones (stem_async=0)
@pytest.mark.parametrize("kt,cout,T,pair,perm,roll", [(5, 8, 6, "1", "1", "1"), (5, 8, 5, "1", "1", "1"),
                                                      (5, 8, 8, "1", "1", "1"), (5, 8, 7, "1", "1", "1"),
                                                      (5, 8, 7, "1", "1", "0"), (5, 8, 7, "1", "1", "s"),
                                                      (5, 8, 6, "0", "1", "1"),
                                                      (1, 64, 6, "1", "1", "1"), (1, 64, 6, "1", "0", "1"),
                                                      (1, 64, 6, "1", "1", "s"),
                                                      (1, 32, 3, "1", "1", "1")])
def test_stem_s2d_fwd_wgrad(kt, cout, T, pair, perm, roll, monkeypatch):
    from pytorchvideo_accelerate_amd.models.fused import to_s2d
    from pytorchvideo_accelerate_amd.ops._ext import require
    monkeypatch.setenv("PVA_ARMS", f"stem_pair={pair},stem_perm={perm},stem_roll={0 if roll == '0' else 1},"
                                   f"stem_async={0 if roll == 's' else 1}")
    C = require()
    g = torch.Generator(device="cpu").manual_seed(7)
    N, H = 2, 40
    x = torch.randn(N, 3, T, H, H, generator=g).to(DEV).to(torch.bfloat16).float()
    w = (torch.randn(cout, 3, kt, 7, 7, generator=g) * 0.05).to(DEV).to(torch.bfloat16).float()
    ref = torch.nn.functional.conv3d(x, w, None, (1, 2, 2), (kt // 2, 3, 3))
    xs = to_s2d(x)
    cpad = (cout + 15) // 16 * 16
    wp = torch.zeros(cpad * kt * 256, device=DEV, dtype=torch.bfloat16)
    C.stem_pack(w.contiguous(), wp, cout, kt)
    M = xs.M
    y = torch.empty(M, cout, device=DEV, dtype=torch.bfloat16)
    tiles = C.stem_tiles(xs.H, xs.W, N)
    stats = torch.empty(tiles, 2, cout, device=DEV)
    C.stem_fwd(xs.t, wp, y, stats, [N, T, xs.H, xs.W], cout, kt)
    got = y.float().reshape(N, T, xs.H, xs.W, cout).permute(0, 4, 1, 2, 3)
    assert rel_err(got, ref) < 1e-2
    yf = y.float()
    torch.testing.assert_close(stats.sum(0)[0], yf.sum(0), rtol=1e-3, atol=1e-2)
    # wgrad
    wr = w.clone().requires_grad_(True)
    out = torch.nn.functional.conv3d(x, wr, None, (1, 2, 2), (kt // 2, 3, 3))
    gy = torch.randn_like(out).to(torch.bfloat16).float()
    out.backward(gy)
    dy = gy.permute(0, 2, 3, 4, 1).reshape(M, cout).contiguous().to(torch.bfloat16)
    acc = torch.zeros(cout * kt * 256, device=DEV)
    grad = torch.zeros_like(w)
    C.stem_wgrad(xs.t, dy, acc, [N, T, xs.H, xs.W], cout, kt)
    C.stem_wgrad_convert(acc, grad, cout, kt, 0.0)
    assert rel_err(grad, wr.grad) < 1e-2
    assert acc.abs().max().item() == 0.0  # re-zeroed for the next use


# LDS-DMA staged uniform-tap loader (ops/tune.DMA): every tile variant x BK, forward (no input affine),
# strided dgrad phases and the backward-BN dgrad epilogue, against PyTorch
DMA_CASES = [CASES[0], CASES[1], CASES[2], CASES[3], CASES[4], CASES[10]]


def _dma_cfgs(g):
    from pytorchvideo_accelerate_amd.ops._ext import require
    from pytorchvideo_accelerate_amd.ops.tune import BK64, DMA, EXPLICIT, UT
    C = require()
    out = []
    for v in range(4):
        for bk in (32, 64):
            if C.conv_ut_legal(list(g), 8, bk):
                out.append(EXPLICIT | UT | DMA | v | (BK64 if bk == 64 else 0))
    return out


@pytest.mark.parametrize("case", DMA_CASES)
def test_conv_dma_loader_fwd_dgrad(case):
    from pytorchvideo_accelerate_amd.ops._ext import require
    from pytorchvideo_accelerate_amd.ops.conv import conv_m_tiles, dgrad_phases, fwd_geometry
    C = require()
    x, w, spec = _mk(case, seed=41)
    ref = torch.nn.functional.conv3d(x, w, None, spec.stride, spec.pad)
    wf, wd = pack_weight(w, spec)
    xa = Act.from_ncthw(x)
    To, Ho, Wo = spec.out_dims(xa.T, xa.H, xa.W)
    M = xa.N * To * Ho * Wo
    g = fwd_geometry(spec, xa.N, xa.T, xa.H, xa.W, xa.ld, spec.cout)
    cfgs = _dma_cfgs(g)
    assert cfgs, "uniform-tap loader must be legal for this case"
    for cfg in cfgs:
        y = torch.empty(M, spec.cout, device=DEV, dtype=torch.bfloat16)
        stats = torch.full(((M + 127) // 128, 2, spec.cout), float("nan"), device=DEV)
        C.conv_igemm(xa.t, wf, y, stats, None, None, 0, 0, g, 8, cfg)
        assert rel_err(Act(y, xa.N, To, Ho, Wo).to_ncthw(), ref) < 1e-2, cfg
        tiles = (M + C.conv_cfg_bm(cfg, spec.cout) - 1) // C.conv_cfg_bm(cfg, spec.cout)
        torch.testing.assert_close(stats[:tiles].sum(0)[0], y.float().sum(0), rtol=1e-3,
                                   atol=1e-2 * y.float().abs().sum(0).max().item() / M ** 0.5)
    gy = torch.randn_like(ref).to(torch.bfloat16).float()
    dx_ref = torch.nn.grad.conv3d_input(x.shape, w, gy, spec.stride, spec.pad)
    dy = Act.from_ncthw(gy)
    N, Ci, T, H, W = x.shape
    geo = dgrad_phases(spec, N, (T, H, W), (dy.T, dy.H, dy.W), dy.ld, Ci)
    for cfg in _dma_cfgs(geo[0]):
        out = torch.zeros(N * T * H * W, Ci, device=DEV, dtype=torch.bfloat16)
        for gg in geo:
            if gg[28] == 0:
                continue
            C.conv_igemm(dy.t, wd, out, None, None, None, 0, 0, gg, 8, cfg if C.conv_ut_legal(list(gg), 8, 64 if cfg & 4 else 32) else -1)
        assert rel_err(Act(out, N, T, H, W).to_ncthw(), dx_ref) < 1e-2, cfg


@pytest.mark.parametrize("case", [CASES[0], CASES[1]])
def test_conv_dma_loader_bn_epilogue(case):
    from pytorchvideo_accelerate_amd.ops._ext import require
    from pytorchvideo_accelerate_amd.ops.conv import dgrad_phases
    C = require()
    x, w, spec = _mk(case, seed=42)
    N, Ci, T, H, W = x.shape
    ref_y = torch.nn.functional.conv3d(x, w, None, spec.stride, spec.pad)
    gy = torch.randn_like(ref_y).to(torch.bfloat16).float()
    M = N * T * H * W
    dx_ref = torch.nn.grad.conv3d_input(x.shape, w, gy, spec.stride, spec.pad).permute(0, 2, 3, 4, 1).reshape(M, Ci)
    gen = torch.Generator(device="cpu").manual_seed(43)
    bf = lambda *s: torch.randn(*s, generator=gen).to(torch.bfloat16).to(DEV)
    res, old, y0 = bf(M, Ci), bf(M, Ci), bf(M, Ci) * 2 + 0.5
    mask = torch.rand(M, Ci, generator=gen).to(DEV) > 0.4
    mean0, rstd0 = torch.randn(Ci, device=DEV) * 0.3, torch.rand(Ci, device=DEV) + 0.5
    _, wd = pack_weight(w, spec)
    dy = Act.from_ncthw(gy)
    geo = dgrad_phases(spec, N, (T, H, W), (dy.T, dy.H, dy.W), dy.ld, Ci)
    for cfg in _dma_cfgs(geo[0]):
        out = old.clone()
        part = torch.full(((M + 127) // 128, 3, Ci), float("nan"), device=DEV)
        C.conv_igemm_epi(dy.t, wd, out, 1, geo[0], 8, res, Ci, _bits(mask), y0, mean0, rstd0, None, None, None, part,
                         None, None, cfg)
        v = (dx_ref + old.float() + res.float()) * mask
        assert rel_err(out, v) < 1.5e-2, cfg
        tiles = (M + C.conv_cfg_bm(cfg, Ci) - 1) // C.conv_cfg_bm(cfg, Ci)
        q = out.float()
        torch.testing.assert_close(part[:tiles].sum(0)[0], q.sum(0), rtol=1e-3,
                                   atol=1e-2 * q.abs().sum(0).max().item() / M ** 0.5)


@pytest.mark.parametrize("case", [CASES[0], CASES[1], CASES[4], CASES[10]])
def test_conv_big_tile(case):
    """256x256 tile of 8 waves (tune.BIG), register and LDS-DMA staging, BK 32/64: forward (+ BN partial sums,
    + consumer affine for the register path) and plain dgrad phases."""
    from pytorchvideo_accelerate_amd.ops._ext import require
    from pytorchvideo_accelerate_amd.ops.conv import dgrad_phases, fwd_geometry
    from pytorchvideo_accelerate_amd.ops.tune import BIG, BIG_HALF, BIG_PF, BK64, DMA, EXPLICIT, UT
    C = require()
    x, w, spec = _mk(case, seed=44)
    Ci = spec.cin
    sc = torch.rand(Ci, device=DEV) + 0.5
    sh = torch.randn(Ci, device=DEV) * 0.5
    wf, wd = pack_weight(w, spec)
    xa = Act.from_ncthw(x)
    To, Ho, Wo = spec.out_dims(xa.T, xa.H, xa.W)
    M = xa.N * To * Ho * Wo
    g = fwd_geometry(spec, xa.N, xa.T, xa.H, xa.W, xa.ld, spec.cout)
    xt = torch.relu(x * sc.view(1, Ci, 1, 1, 1) + sh.view(1, Ci, 1, 1, 1))
    refs = {0: torch.nn.functional.conv3d(x, w, None, spec.stride, spec.pad),
            2: torch.nn.functional.conv3d(xt, w, None, spec.stride, spec.pad)}
    ran = 0
    for bk in (32, 64):
        if spec.cout < 256 or not C.conv_ut_legal(g, 8, bk):
            continue
        base = EXPLICIT | BIG | UT | (BK64 if bk == 64 else 0)
        pf = ((base | DMA | BIG_PF, 0), (base | BIG_HALF | DMA | BIG_PF, 0)) if bk == 64 else ()
        for cfg, aff in ((base, 0), (base | DMA, 0), (base, 2)) + pf:
            y = torch.empty(M, spec.cout, device=DEV, dtype=torch.bfloat16)
            stats = torch.full(((M + 255) // 256, 2, spec.cout), float("nan"), device=DEV)
            C.conv_igemm(xa.t, wf, y, stats, sc if aff else None, sh if aff else None, aff, 0, g, 8, cfg)
            assert rel_err(Act(y, xa.N, To, Ho, Wo).to_ncthw(), refs[aff]) < 1e-2, (cfg, aff)
            yf = y.float()
            torch.testing.assert_close(stats.sum(0)[0], yf.sum(0), rtol=1e-3,
                                       atol=1e-2 * yf.abs().sum(0).max().item() / M ** 0.5)
            ran += 1
    gy = torch.randn_like(refs[0]).to(torch.bfloat16).float()
    dx_ref = torch.nn.grad.conv3d_input(x.shape, w, gy, spec.stride, spec.pad)
    dy = Act.from_ncthw(gy)
    N, _, T, H, W = x.shape
    geo = dgrad_phases(spec, N, (T, H, W), (dy.T, dy.H, dy.W), dy.ld, Ci)
    for bk in (32, 64):
        if Ci < 256 or not all(C.conv_ut_legal(list(gg), 8, bk) for gg in geo if gg[28]):
            continue
        cfgs = (EXPLICIT | BIG | UT | (BK64 if bk == 64 else 0), EXPLICIT | BIG | UT | DMA | (BK64 if bk == 64 else 0))
        if bk == 64:   # L2 touch-prefetch of the big tiles (tune.BIG_PF)
            cfgs += (EXPLICIT | BIG | UT | DMA | BK64 | BIG_PF, EXPLICIT | BIG | BIG_HALF | UT | DMA | BK64 | BIG_PF)
        for cfg in cfgs:
            out = torch.zeros(N * T * H * W, Ci, device=DEV, dtype=torch.bfloat16)
            for gg in geo:
                if gg[28]:
                    C.conv_igemm(dy.t, wd, out, None, None, None, 0, 0, gg, 8, cfg)
            assert rel_err(Act(out, N, T, H, W).to_ncthw(), dx_ref) < 1e-2, cfg
            ran += 1
    assert ran > 0


@pytest.mark.parametrize("case", [CASES[1], CASES[10]])
def test_conv_big_tile_bn_epilogue(case):
    """256x256 tile with the backward-BN dgrad epilogue staged in 64-row slices: residual, ReLU bits, accumulate,
    partial sums of v, v*xhat0, v*xhat1 (register and LDS-DMA loaders, BK 32/64)."""
    from pytorchvideo_accelerate_amd.ops._ext import require
    from pytorchvideo_accelerate_amd.ops.conv import dgrad_phases
    from pytorchvideo_accelerate_amd.ops.tune import BIG, BIG_HALF, BIG_PF, BK64, DMA, EXPLICIT, UT
    C = require()
    x, w, spec = _mk(case, seed=45)
    N, Ci, T, H, W = x.shape
    ref_y = torch.nn.functional.conv3d(x, w, None, spec.stride, spec.pad)
    gy = torch.randn_like(ref_y).to(torch.bfloat16).float()
    M = N * T * H * W
    dx_ref = torch.nn.grad.conv3d_input(x.shape, w, gy, spec.stride, spec.pad).permute(0, 2, 3, 4, 1).reshape(M, Ci)
    gen = torch.Generator(device="cpu").manual_seed(46)
    bf = lambda *s: torch.randn(*s, generator=gen).to(torch.bfloat16).to(DEV)
    res, old, y0, y1 = bf(M, Ci), bf(M, Ci), bf(M, Ci) * 2 + 0.5, bf(M, Ci)
    mask = torch.rand(M, Ci, generator=gen).to(DEV) > 0.4
    mean0, rstd0 = torch.randn(Ci, device=DEV) * 0.3, torch.rand(Ci, device=DEV) + 0.5
    mean1, rstd1 = torch.randn(Ci, device=DEV) * 0.3, torch.rand(Ci, device=DEV) + 0.5
    _, wd = pack_weight(w, spec)
    dy = Act.from_ncthw(gy)
    geo = dgrad_phases(spec, N, (T, H, W), (dy.T, dy.H, dy.W), dy.ld, Ci)
    assert len(geo) == 1
    ran = 0
    for bk in (32, 64):
        if not C.conv_ut_legal(list(geo[0]), 8, bk):
            continue
        base = EXPLICIT | BIG | UT | (BK64 if bk == 64 else 0)
        pf = (base | DMA | BIG_PF, base | BIG_HALF | DMA | BIG_PF) if bk == 64 else ()
        for cfg in (base, base | DMA) + pf:
            out = old.clone()
            part = torch.full(((M + 255) // 256, 3, Ci), float("nan"), device=DEV)
            C.conv_igemm_epi(dy.t, wd, out, 1, geo[0], 8, res, Ci, _bits(mask), y0, mean0, rstd0, y1, mean1, rstd1,
                             part, None, None, cfg)
            v = (dx_ref + old.float() + res.float()) * mask
            assert rel_err(out, v) < 1.5e-2, cfg
            q = out.float()
            s = part.sum(0)
            tol = 2e-2 * (q.abs() * (y0.float() - mean0).abs() * rstd0).sum(0).max().item() / M ** 0.5
            torch.testing.assert_close(s[0], q.sum(0), rtol=1e-3, atol=1e-2 * q.abs().sum(0).max().item() / M ** 0.5)
            torch.testing.assert_close(s[1], (q * (y0.float() - mean0) * rstd0).sum(0), rtol=1e-3, atol=tol)
            torch.testing.assert_close(s[2], (q * (y1.float() - mean1) * rstd1).sum(0), rtol=1e-3, atol=tol)
            ran += 1
    assert ran > 0


HALO_CASES = [CASES[2], CASES[6], CASES[8], (16, 16, (1, 3, 3), (1, 1, 1), (0, 1, 1), (2, 3, 9, 13)),
              (32, 8, (3, 1, 1), (1, 1, 1), (1, 0, 0), (2, 5, 7, 9)), (8, 8, (1, 3, 3), (1, 1, 1), (0, 1, 1), (1, 4, 17, 11)),
              (128, 128, (1, 3, 3), (1, 1, 1), (0, 1, 1), (1, 2, 10, 12)), (64, 64, (3, 1, 1), (1, 1, 1), (1, 0, 0), (1, 6, 5, 7)),
              (32, 32, (1, 3, 3), (1, 1, 1), (0, 1, 1), (2, 2, 14, 14))]


@pytest.mark.parametrize("case", HALO_CASES)
@pytest.mark.parametrize("affine", [False, True])
@pytest.mark.parametrize("option", [0, 1])
def test_conv_wgrad_halo(case, affine, option):
    """Halo-staged weight gradient (stride-1 'same' convs): box wrap across rows and frames, partial boxes at
    the T / H edges, padding taps, Cout < 16, k-tile groups, BN-ReLU recompute of the input."""
    from pytorchvideo_accelerate_amd.ops.conv import HALO, halo_wgrad_plan
    x, w, spec = _mk(case, seed=51)
    C = spec.cin
    sc = torch.rand(C, device=DEV) + 0.5
    sh = torch.randn(C, device=DEV) * 0.5
    xt = torch.relu(x * sc.view(1, C, 1, 1, 1) + sh.view(1, C, 1, 1, 1)) if affine else x
    xt = xt.to(torch.bfloat16).float()
    w.requires_grad_(True)
    ref_y = torch.nn.functional.conv3d(xt, w, None, spec.stride, spec.pad)
    gy = torch.randn_like(ref_y).to(torch.bfloat16).float()
    ref_y.backward(gy)
    dy = Act.from_ncthw(gy)
    assert halo_wgrad_plan(spec, dy.M, (dy.T, dy.H, dy.W), option) is not None
    grad = torch.zeros_like(w)
    conv_wgrad(dy, Act.from_ncthw(x), spec, grad, in_scale=sc if affine else None,
               in_shift=sh if affine else None, variant=HALO | option)
    assert rel_err(grad, w.grad) < 1.5e-2
