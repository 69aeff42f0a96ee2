"""Direct fp32 unit tests of the BatchNorm / pooling kernels (csrc/kernels/bn_eltwise.hip) at edge shapes:
C = 8 / 16 / 24 channels, odd row counts and odd H / W.  Each is compared against a float64 / float32 PyTorch
reference of the same op (BatchNorm training-mode statistics and running-stat update, the BN backward
reduce -> finalize -> apply chain with every mask mode, the stem's BN+ReLU+maxpool(3, s2, p1) forward and its
argmax-gather backward, AvgPool3d(stride 1) forward / backward at a channel offset of a wider output)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _C():
    from pytorchvideo_accelerate_amd.ops._ext import require
    return require()


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


def _bits(mask):
    M, C = mask.shape
    w = (1 << torch.arange(8, device=mask.device)).to(torch.int32)
    return (mask.view(M, C // 8, 8).to(torch.int32) * w).sum(-1).to(torch.uint8)


@pytest.mark.parametrize("C,tiles,count", [(8, 5, 1001), (16, 37, 4097), (24, 1, 2)])
def test_bn_finalize_running_stats(C, tiles, count):
    K = _C()
    g = torch.Generator().manual_seed(C)
    x = torch.randn(count, C, generator=g, dtype=torch.float64) * 2 + 0.7
    # split the rows over `tiles` partial slabs [tiles][2][C] (sum, sum of squares)
    idx = torch.arange(count) % tiles
    part = torch.zeros(tiles, 2, C, dtype=torch.float64)
    part[:, 0].index_add_(0, idx, x)
    part[:, 1].index_add_(0, idx, x * x)
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g)
    rm0, rv0 = torch.randn(C, generator=g), torch.rand(C, generator=g) + 0.5
    rm, rv = rm0.clone().to(DEV), rv0.clone().to(DEV)
    nbt = torch.zeros((), dtype=torch.long, device=DEV)
    mean, rstd, scale, shift = (torch.empty(C, device=DEV) for _ in range(4))
    K.bn_finalize(part.float().to(DEV), tiles, C, count, gamma.to(DEV), beta.to(DEV), rm, rv, nbt, 0.1, 1e-5,
                  mean, rstd, scale, shift)
    torch.cuda.synchronize()
    mu, var = x.mean(0), x.var(0, unbiased=False)
    r = 1 / (var + 1e-5).sqrt()
    assert _rel(mean.cpu(), mu) < 1e-5 and _rel(rstd.cpu(), r) < 1e-5
    assert _rel(scale.cpu(), gamma.double() * r) < 1e-5
    assert _rel(shift.cpu(), beta.double() - mu * gamma.double() * r) < 1e-5
    unb = x.var(0, unbiased=True) if count > 1 else var
    assert _rel(rm.cpu(), 0.9 * rm0.double() + 0.1 * mu) < 1e-5
    assert _rel(rv.cpu(), 0.9 * rv0.double() + 0.1 * unb) < 1e-5
    assert int(nbt) == 1


@pytest.mark.parametrize("C,M", [(8, 1001), (16, 777), (24, 4099)])
@pytest.mark.parametrize("mask_mode", [3, 2, 0])
def test_bn_backward_chain(C, M, mask_mode):
    """bn_bwd_reduce -> bn_bwd_finalize -> bn_bwd_apply vs autograd of training-mode BatchNorm (+ReLU mask)."""
    K = _C()
    g = torch.Generator().manual_seed(C * 10 + mask_mode)
    y = (torch.randn(M, C, generator=g) * 1.5 + 0.3).to(torch.bfloat16)
    dout = torch.randn(M, C, generator=g).to(torch.bfloat16)
    gamma = torch.rand(C, generator=g) + 0.5
    yf = y.double()
    mu, var = yf.mean(0), yf.var(0, unbiased=False)
    rstd = 1 / (var + 1e-5).sqrt()
    ms, mh = torch.rand(C, generator=g) + 0.2, torch.randn(C, generator=g) * 0.5
    maskb = torch.rand(M, C, generator=g) > 0.3
    if mask_mode == 3:
        m = maskb
    elif mask_mode == 2:
        m = (y.float() * ms + mh) > 0
    else:
        m = torch.ones(M, C, dtype=torch.bool)
    dz = dout.double() * m
    # reference: d/dy of sum(dz * BN(y)) with batch statistics
    yr = yf.clone().requires_grad_(True)
    mu_r = yr.mean(0)
    var_r = ((yr - mu_r) ** 2).mean(0)
    z = (yr - mu_r) / (var_r + 1e-5).sqrt() * gamma.double()
    z.backward(dz)
    xhat = (yf - mu) * rstd
    blocks, rpb = K.bn_bwd_blocks(M, C)
    part = torch.full((blocks, 3, C), float("nan"), device=DEV)
    yd, doutd = y.to(DEV), dout.to(DEV)
    mo = _bits(maskb.to(DEV)) if mask_mode == 3 else None
    msd, mhd = (ms.to(DEV), mh.to(DEV)) if mask_mode == 2 else (None, None)
    mean_d, rstd_d = mu.float().to(DEV), rstd.float().to(DEV)
    dzw = torch.full((M, C + 8), 5.0, dtype=torch.bfloat16, device=DEV)   # masked dz written by the same pass
    K.bn_bwd_reduce(doutd, C, mask_mode, mo, C // 8, msd, mhd, yd, mean_d, rstd_d, None, None, None, M, C, blocks,
                    rpb, part, dzw, C + 8)
    assert torch.equal(dzw[:, :C].cpu().double(), dz) and torch.all(dzw[:, C:] == 5.0)
    dgamma, dbeta = torch.full((C,), 2.0, device=DEV), torch.full((C,), 3.0, device=DEV)
    coef = torch.empty(3 * C, device=DEV)
    K.bn_bwd_finalize(part, blocks, C, M, 0, gamma.to(DEV), mean_d, rstd_d, dgamma, dbeta, 0.5, coef)
    dy = torch.empty(M, C, dtype=torch.bfloat16, device=DEV)
    dzbuf = torch.randn(M, C, generator=g).to(torch.bfloat16)
    dzout = dzbuf.to(DEV)
    K.bn_bwd_apply(doutd, C, mask_mode, mo, C // 8, msd, mhd, yd, coef, dy, None, None, None, dzout, C, 1, M, C)
    torch.cuda.synchronize()
    assert _rel(dbeta.cpu(), 1.5 + dz.sum(0)) < 1e-5                     # beta_acc = 0.5 onto 3.0
    assert _rel(dgamma.cpu(), 1.0 + (dz * xhat).sum(0)) < 1e-4
    assert _rel(dy.cpu(), yr.grad) < 1e-2
    assert _rel(dzout.cpu(), dzbuf.double() + dz) < 1e-2                  # dz accumulated into dzout


@pytest.mark.parametrize("C,H,W", [(8, 15, 13), (16, 9, 11), (24, 8, 7)])
def test_stem_pool_fwd_bwd(C, H, W):
    K = _C()
    NT = 3
    g = torch.Generator().manual_seed(C + H)
    y = torch.randn(NT * H * W, C, generator=g).to(torch.bfloat16)
    sc = torch.rand(C, generator=g) + 0.5
    sh = torch.randn(C, generator=g) * 0.2 + 0.5
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    ldo = C + 8
    out = torch.zeros(NT * Ho * Wo, ldo, dtype=torch.bfloat16, device=DEV)
    arg = torch.empty(NT * Ho * Wo * C, dtype=torch.uint8, device=DEV)
    K.stem_pool_fwd(y.to(DEV), sc.to(DEV), sh.to(DEV), out, ldo, arg, NT, H, W, Ho, Wo, C)
    a = torch.relu(y.float() * sc + sh).view(NT, H, W, C).permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    ref = F.max_pool2d(a, 3, 2, 1)
    assert ref.shape[-2:] == (Ho, Wo)
    got = out[:, :C].float().cpu().view(NT, Ho, Wo, C).permute(0, 3, 1, 2)
    assert _rel(got, ref.detach()) < 5e-3
    assert torch.all(out[:, C:] == 0)
    dout = torch.randn(NT * Ho * Wo, ldo, generator=g).to(torch.bfloat16)
    dact = torch.empty(NT * H * W, C, dtype=torch.bfloat16, device=DEV)
    K.stem_pool_bwd(dout.to(DEV), ldo, arg, dact, NT, H, W, Ho, Wo, C)
    torch.cuda.synchronize()
    ref.backward(dout[:, :C].float().view(NT, Ho, Wo, C).permute(0, 3, 1, 2))
    want = a.grad.permute(0, 2, 3, 1).reshape(NT * H * W, C)
    assert _rel(dact.cpu(), want) < 1e-2


@pytest.mark.parametrize("dims,k", [((2, 3, 7, 5, 16), (2, 3, 3)), ((1, 4, 9, 9, 8), (4, 9, 9)),
                                    ((3, 2, 5, 7, 24), (1, 2, 3)), ((5, 8, 7, 7, 2048), (8, 7, 7)),
                                    ((3, 32, 7, 7, 256), (32, 7, 7)), ((2, 3, 5, 5, 40), (3, 5, 5))])
def test_avgpool_fwd_bwd(dims, k):
    K = _C()
    N, T, H, W, C = dims
    g = torch.Generator().manual_seed(sum(dims))
    x = torch.randn(N, T, H, W, C, generator=g).to(torch.bfloat16)
    To, Ho, Wo = T - k[0] + 1, H - k[1] + 1, W - k[2] + 1
    P = To * Ho * Wo
    coff, ldo = 8, C + 16
    out = torch.full((N * P, ldo), 7.0, device=DEV)
    K.avgpool_fwd(x.to(DEV), [N, T, H, W, C], list(k), out, ldo, coff)
    xr = x.float().permute(0, 4, 1, 2, 3).contiguous().requires_grad_(True)
    ref = F.avg_pool3d(xr, k, stride=1)
    got = out[:, coff:coff + C].cpu().view(N, To, Ho, Wo, C).permute(0, 4, 1, 2, 3)
    assert _rel(got, ref.detach()) < 1e-5
    assert torch.all(out[:, :coff] == 7.0) and torch.all(out[:, coff + C:] == 7.0)
    dout = torch.randn(N * P, ldo, generator=g)
    dx = torch.empty(N * T * H * W, C, dtype=torch.bfloat16, device=DEV)
    K.avgpool_bwd(dout.to(DEV), ldo, coff, [N, T, H, W, C], list(k), dx)
    torch.cuda.synchronize()
    ref.backward(dout[:, coff:coff + C].view(N, To, Ho, Wo, C).permute(0, 4, 1, 2, 3))
    want = xr.grad.permute(0, 2, 3, 4, 1).reshape(-1, C)
    assert _rel(dx.cpu(), want) < 5e-3


@pytest.mark.parametrize("C,H,W", [(8, 15, 13), (64, 12, 9), (16, 8, 7)])
def test_stem_pool_bn_backward_fused(C, H, W):
    """Stem backward on the fused path (pooled-grid BN sums from ``ymax`` + stem_pool_bn_apply) vs float64
    autograd of maxpool(relu(BN_train(y))) — dgamma, dbeta and dy."""
    K = _C()
    NT = 3
    g = torch.Generator().manual_seed(C * 7 + H)
    M = NT * H * W
    y = (torch.randn(M, C, generator=g) * 1.3 + 0.2).to(torch.bfloat16)
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g) * 0.3
    yf = y.double()
    mu, var = yf.mean(0), yf.var(0, unbiased=False)
    rstd = 1 / (var + 1e-5).sqrt()
    scale = (gamma.double() * rstd).float()
    shift = (beta.double() - mu * gamma.double() * rstd).float()
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    P = NT * Ho * Wo
    ldo = C + 8
    out = torch.zeros(P, ldo, dtype=torch.bfloat16, device=DEV)
    arg = torch.empty(P * C, dtype=torch.uint8, device=DEV)
    ymax = torch.empty(P, C, dtype=torch.bfloat16, device=DEV)
    yd = y.to(DEV)
    sc_d, sh_d = scale.to(DEV), shift.to(DEV)
    K.stem_pool_fwd(yd, sc_d, sh_d, out, ldo, arg, NT, H, W, Ho, Wo, C, ymax)
    dout = torch.randn(P, ldo, generator=g).to(torch.bfloat16)
    doutd = dout.to(DEV)
    mean_d, rstd_d = mu.float().to(DEV), rstd.float().to(DEV)
    blocks, rpb = K.bn_bwd_blocks(P, C)
    part = torch.full((blocks, 3, C), float("nan"), device=DEV)
    K.bn_bwd_reduce(doutd, ldo, 2, None, 0, sc_d, sh_d, ymax, mean_d, rstd_d, None, None, None, P, C, blocks, rpb, part)
    dgamma, dbeta = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    coef = torch.empty(3 * C, device=DEV)
    K.bn_bwd_finalize(part, blocks, C, M, 0, gamma.to(DEV), mean_d, rstd_d, dgamma, dbeta, 0.0, coef)
    dy = torch.empty(M, C, dtype=torch.bfloat16, device=DEV)
    K.stem_pool_bn_apply(doutd, ldo, arg, yd, sc_d, sh_d, coef, dy, NT, H, W, Ho, Wo, C)
    torch.cuda.synchronize()
    # float64 reference (BN with batch statistics of y, ReLU, 3x3/s2/p1 max pool)
    yr = yf.clone().requires_grad_(True)
    gr = gamma.double().requires_grad_(True)
    br = beta.double().requires_grad_(True)
    m_r = yr.mean(0)
    v_r = ((yr - m_r) ** 2).mean(0)
    a = torch.relu((yr - m_r) / (v_r + 1e-5).sqrt() * gr + br)
    pooled = F.max_pool2d(a.view(NT, H, W, C).permute(0, 3, 1, 2), 3, 2, 1)
    pooled.backward(dout[:, :C].double().view(NT, Ho, Wo, C).permute(0, 3, 1, 2))
    assert _rel(dbeta.cpu(), br.grad) < 1e-4
    assert _rel(dgamma.cpu(), gr.grad) < 1e-3
    assert _rel(dy.cpu(), yr.grad) < 2e-2


@pytest.mark.parametrize("C,tiles", [(8, 20480), (64, 17920), (256, 1280), (2048, 490), (24, 3)])
def test_two_level_finalize_matches_single_level(C, tiles):
    """The coalesced two-level finalize (fin workspace: partial doubles + self-resetting counters) against the
    one-block-per-channel kernels, forward and backward, repeated (the counters return to zero) at the tile counts
    of the B=160 step (halo 784/224-position tiles, 128-row tiles, few tiles)."""
    K = _C()
    g = torch.Generator().manual_seed(C + tiles)
    part2 = (torch.randn(tiles, 2, C, generator=g) + 0.5).abs().to(DEV)
    part3 = torch.randn(tiles, 3, C, generator=g).to(DEV)
    count = tiles * 100
    gamma, beta = (torch.rand(C, generator=g) + 0.5).to(DEV), torch.randn(C, generator=g).to(DEV)
    fin = torch.zeros(K.fin_doubles(C), dtype=torch.float64, device=DEV)
    ref = [torch.empty(C, device=DEV) for _ in range(4)]
    K.bn_finalize(part2, tiles, C, count, gamma, beta, None, None, None, 0.1, 1e-5, *ref)
    rm_a, rv_a = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    rm_b, rv_b = rm_a.clone(), rv_a.clone()
    K.bn_finalize(part2, tiles, C, count, gamma, beta, rm_a, rv_a, None, 0.1, 1e-5, *[torch.empty(C, device=DEV) for _ in range(4)])
    for rep in range(3):
        out = [torch.full((C,), float("nan"), device=DEV) for _ in range(4)]
        K.bn_finalize(part2, tiles, C, count, gamma, beta, None, None, None, 0.1, 1e-5, *out, fin)
        for a, b in zip(out, ref):
            torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)
    K.bn_finalize(part2, tiles, C, count, gamma, beta, rm_b, rv_b, None, 0.1, 1e-5, *[torch.empty(C, device=DEV) for _ in range(4)], fin)
    torch.testing.assert_close(rm_b, rm_a, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(rv_b, rv_a, rtol=1e-6, atol=1e-7)
    mean, rstd = torch.randn(C, device=DEV), torch.rand(C, device=DEV) + 0.5
    for which in (0, 1):
        cr, dgr, dbr = torch.empty(3 * C, device=DEV), torch.ones(C, device=DEV), torch.ones(C, device=DEV)
        K.bn_bwd_finalize(part3, tiles, C, count, which, gamma, mean, rstd, dgr, dbr, 0.5, cr)
        for rep in range(2):
            c2, dg2, db2 = torch.empty(3 * C, device=DEV), torch.ones(C, device=DEV), torch.ones(C, device=DEV)
            K.bn_bwd_finalize(part3, tiles, C, count, which, gamma, mean, rstd, dg2, db2, 0.5, c2, fin)
            torch.testing.assert_close(c2, cr, rtol=1e-5, atol=1e-7)
            torch.testing.assert_close(dg2, dgr, rtol=1e-5, atol=1e-6)
            torch.testing.assert_close(db2, dbr, rtol=1e-5, atol=1e-6)
    ctr = fin[256 * 2 * C:].view(torch.int32)[: (C + 63) // 64]
    assert torch.all(ctr == 0), ctr   # every counter reset by its last workgroup
