"""BatchNorm folding of a bottleneck's 1x1 conv_c (csrc/kernels/bn_fold.hip + the Gram mode of the wgrad kernel +
the fused residual-output epilogue of conv_igemm) against float64 PyTorch references of the same math:

  a = relu(yb * sb + hb) (bf16, as the conv consumes it), yc = a Wc^T, out = relu(BN_c(yc) + r)
  forward statistics from Ga = a^T a and s = 1^T a; backward dWc, dgamma, dbeta, d a from G = dz^T a.
"""
import pytest
import torch

from pytorchvideo_accelerate_amd.ops.conv import ConvSpec, fwd_geometry, pack_weight, wgrad_splits

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _C():
    from pytorchvideo_accelerate_amd.ops._ext import require
    return require()


def _data(M, c, Co, seed=0):
    g = torch.Generator().manual_seed(seed)
    yb = torch.randn(M, c, generator=g).to(torch.bfloat16).to(DEV)
    sb = (torch.rand(c, generator=g) + 0.5).to(DEV)
    hb = (torch.randn(c, generator=g) * 0.3).to(DEV)
    w = (torch.randn(Co, c, 1, 1, 1, generator=g) * (2.0 / c) ** 0.5).to(DEV)
    a = torch.relu(yb.float() * sb + hb).to(torch.bfloat16).double()     # operand values the kernels multiply
    return g, yb, sb, hb, w, a


def _gram(yb, sb, hb, c, N=1, T=1, H=None, W=None):
    C = _C()
    M = yb.shape[0]
    H = H or M
    W = W or 1
    spec = ConvSpec(c, c, (1, 1, 1))
    splits, pps = wgrad_splits(M, c, c)
    acc = torch.zeros(c * c, device=DEV)
    colsum = torch.zeros(splits * c, device=DEV)
    g = [M, c, c, c, c, c, T, H, W, T, H, W, 1, 1, 1, 1, 1, 1, 0, 0, 0, splits, pps]
    C.conv_wgrad(yb, yb, acc, sb, hb, 2, g, 8, 0, -1, 1, colsum)
    Ga = torch.empty(c, c, device=DEV)
    C.wgrad_reduce(acc, Ga, splits, c, 1, c, c, 1.0, 0.0, 0)
    return Ga, colsum, splits


@pytest.mark.parametrize("M,c", [(1000, 64), (4096, 128), (777, 8)])
def test_gram_mode(M, c):
    _, yb, sb, hb, _, a = _data(M, c, 4 * c)
    Ga, colsum, splits = _gram(yb, sb, hb, c)
    torch.cuda.synchronize()
    ref = a.t() @ a
    assert ((Ga.double().cpu() - ref.cpu()).norm() / ref.norm()).item() < 1e-5
    s = colsum.view(splits, c).sum(0).double().cpu()
    assert ((s - a.sum(0).cpu()).norm() / a.sum(0).norm()).item() < 1e-5


@pytest.mark.parametrize("identity", [True, False])
def test_fres_epilogue(identity):
    C = _C()
    N, T, H, W, c, Co = 2, 2, 8, 8, 64, 256
    M = N * T * H * W
    g, yb, sb, hb, w, a = _data(M, c, Co, seed=1)
    spec = ConvSpec(c, Co, (1, 1, 1))
    wf, _ = pack_weight(w, spec)
    fsc = (torch.rand(Co, generator=g) + 0.5).to(DEV)
    fsh = (torch.randn(Co, generator=g) * 0.2).to(DEV)
    # residual as a channel slice of a wider buffer (the concat case)
    resbuf = torch.randn(M, Co + 32, generator=g).to(torch.bfloat16).to(DEV)
    res = resbuf[:, :Co]
    rsc = None if identity else (torch.rand(Co, generator=g) + 0.5).to(DEV)
    rsh = None if identity else (torch.randn(Co, generator=g) * 0.2).to(DEV)
    outbuf = torch.zeros(M, Co + 16, dtype=torch.bfloat16, device=DEV)
    out = outbuf[:, :Co]
    mask = torch.zeros(M, Co // 8, dtype=torch.uint8, device=DEV)
    geo = fwd_geometry(spec, N, T, H, W, c, out.stride(0))
    C.conv_igemm_fres(yb, wf, out, sb, hb, 2, geo, 8, -1, fsc, fsh, res, res.stride(0), rsc, rsh, mask)
    torch.cuda.synchronize()
    yc = a @ w.view(Co, c).to(torch.bfloat16).double().t()
    r = res.double() if identity else res.double() * rsc.double() + rsh.double()
    ref = torch.relu(yc * fsc.double() + fsh.double() + r)
    err = ((out.double() - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err
    bits = (out.float() > 0).view(M, Co // 8, 8).to(torch.int32)
    want = (bits * (2 ** torch.arange(8, device=DEV, dtype=torch.int32))).sum(-1).to(torch.uint8)
    assert torch.equal(mask, want)
    assert torch.all(outbuf[:, Co:] == 0)


@pytest.mark.parametrize("M,c,Co", [(2048, 64, 256), (1000, 128, 512)])
def test_bnfold_forward_stats_and_backward(M, c, Co):
    C = _C()
    g, yb, sb, hb, w, a = _data(M, c, Co, seed=2)
    spec = ConvSpec(c, Co, (1, 1, 1))
    wf, wd = pack_weight(w, spec)
    Wc = w.view(Co, c).to(torch.bfloat16).double()
    gamma = (torch.rand(Co, generator=g) + 0.5).to(DEV)
    beta = (torch.randn(Co, generator=g) * 0.1).to(DEV)
    rm, rv = torch.zeros(Co, device=DEV), torch.ones(Co, device=DEV)
    nbt = torch.zeros((), dtype=torch.long, device=DEV)
    Ga, colsum, splits = _gram(yb, sb, hb, c)
    T = torch.empty(Co, c, device=DEV)
    s = torch.empty(c, device=DEV)
    mean, rstd = torch.empty(Co, device=DEV), torch.empty(Co, device=DEV)
    scale, shift = torch.empty(Co, device=DEV), torch.empty(Co, device=DEV)
    C.bnfold_fwd_stats(wf, Ga, colsum, splits, Co, c, M, T, s, gamma, beta, rm, rv, nbt, 0.1, 1e-5, mean, rstd,
                       scale, shift)
    torch.cuda.synchronize()
    yc = a @ Wc.t()
    mu, var = yc.mean(0), yc.var(0, unbiased=False)
    rel = lambda x, y: ((x.double().cpu() - y.cpu()).norm() / y.norm().clamp_min(1e-30)).item()
    assert rel(mean, mu) < 1e-4 and rel(rstd, 1 / (var + 1e-5).sqrt()) < 1e-4
    assert rel(rv, 0.9 + 0.1 * yc.var(0, unbiased=True)) < 1e-4 and int(nbt) == 1
    # ---- backward ----
    # dz with a large per-channel mean (the avg-pooled head gradient is spatially constant): the BN backward
    # removes it, so the fold's mean corrections must cancel before any bf16 rounding
    dz = (torch.randn(M, Co, generator=g) * 0.1 + torch.randn(1, Co, generator=g) * 3).to(torch.bfloat16).to(DEV)
    part = torch.zeros(1, 3, Co, device=DEV)
    part[0, 0] = dz.float().sum(0)
    G = torch.empty(Co, c, device=DEV)
    splits2, pps2 = wgrad_splits(M, Co, c)
    acc = torch.zeros(Co * c, device=DEV)
    g2 = [M, Co, c, c, Co, c, 1, M, 1, 1, M, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, splits2, pps2]
    C.conv_wgrad(dz, yb, acc, sb, hb, 2, g2, 8, 0, -1)
    C.wgrad_reduce(acc, G, splits2, Co, 1, c, c, 1.0, 0.0, 0)
    dgam, dbet = torch.zeros(Co, device=DEV), torch.zeros(Co, device=DEV)
    dW = torch.zeros(Co, c, device=DEV)
    coef = torch.empty(4 * Co, device=DEV)
    W1t = torch.empty(c, Co, dtype=torch.bfloat16, device=DEV)
    W2 = torch.empty(c, c, dtype=torch.bfloat16, device=DEV)
    bias = torch.empty(2 * c, device=DEV)
    C.bnfold_bwd(part, 1, wf, wd, G, T, s, Co, c, M, gamma, mean, rstd, dgam, dbet, dW, 0.0, coef, W1t, W2, bias)
    # d act = a W2 + bias (fwd conv, affine fold) then += dz W1 (dgrad)
    dact = torch.empty(M, c, dtype=torch.bfloat16, device=DEV)
    gspec = ConvSpec(c, c, (1, 1, 1))
    C.conv_igemm(yb, W2, dact, None, sb, hb, 2, 0, fwd_geometry(gspec, 1, 1, M, 1, c, c), 8, -1, bias[c:])
    from pytorchvideo_accelerate_amd.ops.conv import dgrad_phases
    for gd in dgrad_phases(spec, 1, (1, M, 1), (1, M, 1), Co, c):
        C.conv_igemm_epi(dz, W1t, dact, 1, gd, 8, None, 0, None, None, None, None, None, None, None, None, None,
                         None, -1, bias[:c])
    torch.cuda.synchronize()
    # fp64 reference of BN backward + conv_c backward
    xhat = (yc - mu) / (var + 1e-5).sqrt()
    dzd = dz.double()
    dbeta_r, dgam_r = dzd.sum(0), (dzd * xhat).sum(0)
    r = 1 / (var + 1e-5).sqrt()
    dyc = gamma.double() * r / M * (M * dzd - dbeta_r - xhat * dgam_r)
    assert rel(dbet, dbeta_r) < 1e-4 and rel(dgam, dgam_r) < 1e-3
    assert rel(dW, dyc.t() @ a) < 2e-3
    err = rel(dact, dyc @ Wc)
    assert err < 2e-2, err
