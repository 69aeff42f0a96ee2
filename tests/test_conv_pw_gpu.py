"""Streaming pointwise conv kernel (csrc/kernels/conv_pw.hip, autotuner word ``tune.PW``) against float64
PyTorch references of the same op: forward with the consumer-side BN(+ReLU) on the input, bias, accumulate and
the forward BN partial sums; the BN-folded residual-unit output (fres); the dgrad backward-BN epilogue
(residual, ReLU bits / BN-affine mask, bias, accumulate, partial sums of v, v*xhat0, v*xhat1).  Odd row
counts, K not a multiple of 32, channel-slice inputs/outputs (row strides wider than the channel count)."""
import pytest
import torch

from pytorchvideo_accelerate_amd.ops.conv import ConvSpec, dgrad_phases, fwd_geometry, pack_weight

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _C():
    from pytorchvideo_accelerate_amd.ops._ext import require
    return require()


def _cfgs():
    from pytorchvideo_accelerate_amd.ops.tune import EXPLICIT, PW, PW_ROWS, PW_W4
    return [EXPLICIT | PW | w | v for w in (0, PW_W4) for v in range(len(PW_ROWS))]


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


def _bits(mask):
    M, C = mask.shape
    w = (1 << torch.arange(8, device=mask.device)).to(torch.int32)
    return (mask.view(M, C // 8, 8).to(torch.int32) * w).sum(-1).to(torch.uint8)


# (M as (N, T, H, W), Cin, Cout, extra input / output row padding)
FWD = [((2, 3, 7, 9), 64, 256, 0, 0), ((1, 4, 10, 10), 128, 512, 16, 8), ((3, 1, 11, 13), 8, 32, 8, 0),
       ((2, 2, 9, 9), 80, 256, 0, 16), ((1, 2, 15, 15), 256, 64, 0, 0), ((1, 1, 33, 31), 200, 96, 8, 0),
       ((2, 4, 8, 8), 32, 128, 0, 0), ((1, 2, 7, 9), 256, 1024, 0, 0), ((1, 3, 5, 7), 64, 2048, 0, 0)]


@pytest.mark.parametrize("case", FWD)
@pytest.mark.parametrize("aff", [0, 1, 2])
def test_pw_forward(case, aff):
    C = _C()
    (N, T, H, W), ci, co, xpad, ypad = case
    M = N * T * H * W
    g = torch.Generator().manual_seed(ci * 7 + co + aff)
    spec = ConvSpec(ci, co, (1, 1, 1))
    w = torch.randn(co, ci, 1, 1, 1, generator=g) * (2.0 / ci) ** 0.5
    wf, _ = pack_weight(w.to(DEV), spec)
    xbuf = torch.randn(M, ci + xpad, generator=g).to(torch.bfloat16).to(DEV)
    x = xbuf[:, :ci]
    sc = (torch.rand(ci, generator=g) + 0.5).to(DEV)
    sh = (torch.randn(ci, generator=g) * 0.3).to(DEV)
    bias = (torch.randn(co, generator=g) * 0.2).to(DEV)
    xin = x.double()
    if aff:
        xin = x.float() * sc + sh
        xin = (torch.relu(xin) if aff == 2 else xin).to(torch.bfloat16).double()
    ref0 = xin @ w.view(co, ci).to(torch.bfloat16).double().t().to(DEV)
    geo = fwd_geometry(spec, N, T, H, W, xbuf.stride(0), co + ypad)
    assert C.conv_pw_legal(list(geo), 8)
    for cfg in _cfgs():
        for accum, use_bias in ((0, False), (1, True)):
            ybuf = torch.randn(M, co + ypad, generator=g).to(torch.bfloat16).to(DEV)
            old = ybuf.clone()
            y = ybuf[:, :co]
            rows = C.conv_cfg_bm(cfg, co)
            tiles = (M + rows - 1) // rows
            stats = torch.full((tiles, 2, co), float("nan"), device=DEV)
            C.conv_igemm(x, wf, y, stats, sc if aff else None, sh if aff else None, aff, accum, list(geo), 8, cfg,
                         bias if use_bias else None)
            torch.cuda.synchronize()
            ref = ref0 + (bias.double() if use_bias else 0) + (old[:, :co].double() if accum else 0)
            assert _rel(y, ref) < 8e-3, (cfg, accum)
            assert torch.equal(ybuf[:, co:], old[:, co:]), "wrote outside the channel slice"
            q = y.double()
            s = stats.double().sum(0)
            assert _rel(s[0], q.sum(0)) < 1e-4 and _rel(s[1], (q * q).sum(0)) < 1e-4, cfg


@pytest.mark.parametrize("identity", [True, False])
@pytest.mark.parametrize("shape", [((2, 2, 8, 8), 64, 256), ((1, 3, 9, 11), 128, 512), ((2, 1, 7, 7), 16, 64),
                                   ((1, 2, 7, 9), 256, 1024)])
def test_pw_fres(identity, shape):
    C = _C()
    (N, T, H, W), c, Co = shape
    M = N * T * H * W
    g = torch.Generator().manual_seed(Co + identity)
    spec = ConvSpec(c, Co, (1, 1, 1))
    w = torch.randn(Co, c, 1, 1, 1, generator=g) * (2.0 / c) ** 0.5
    wf, _ = pack_weight(w.to(DEV), spec)
    yb = torch.randn(M, c, generator=g).to(torch.bfloat16).to(DEV)
    sb = (torch.rand(c, generator=g) + 0.5).to(DEV)
    hb = (torch.randn(c, generator=g) * 0.3).to(DEV)
    a = torch.relu(yb.float() * sb + hb).to(torch.bfloat16).double()
    fsc = (torch.rand(Co, generator=g) + 0.5).to(DEV)
    fsh = (torch.randn(Co, generator=g) * 0.2).to(DEV)
    resbuf = torch.randn(M, Co + 32, generator=g).to(torch.bfloat16).to(DEV)
    res = resbuf[:, :Co]
    rsc = None if identity else (torch.rand(Co, generator=g) + 0.5).to(DEV)
    rsh = None if identity else (torch.randn(Co, generator=g) * 0.2).to(DEV)
    yc = a @ w.view(Co, c).to(torch.bfloat16).double().t().to(DEV)
    r = res.double() if identity else res.double() * rsc.double() + rsh.double()
    ref = torch.relu(yc * fsc.double() + fsh.double() + r)
    geo = fwd_geometry(spec, N, T, H, W, c, Co + 16)
    for cfg in _cfgs():
        outbuf = torch.zeros(M, Co + 16, dtype=torch.bfloat16, device=DEV)
        out = outbuf[:, :Co]
        mask = torch.zeros(M, Co // 8, dtype=torch.uint8, device=DEV)
        C.conv_igemm_fres(yb, wf, out, sb, hb, 2, list(geo), 8, cfg, fsc, fsh, res, res.stride(0), rsc, rsh, mask)
        torch.cuda.synchronize()
        assert _rel(out, ref) < 1e-2, cfg
        assert torch.equal(mask, _bits(out.float() > 0)), cfg
        assert torch.all(outbuf[:, Co:] == 0)


@pytest.mark.parametrize("shape", [((2, 3, 7, 9), 256, 64), ((1, 2, 10, 10), 64, 256), ((2, 2, 9, 7), 512, 128),
                                   ((1, 1, 13, 13), 32, 24), ((1, 2, 7, 9), 1024, 256)])
@pytest.mark.parametrize("mode", ["res_mask_dual_accum", "bnmask_bias", "plain"])
def test_pw_dgrad_epilogue(shape, mode):
    """dx = dy W for a 1x1 conv Ci -> Co (K = Co, N = Ci) with the backward-BN epilogue."""
    C = _C()
    (N, T, H, W), ci, co = shape
    if co > 256:
        pytest.skip("K > 256: not a pointwise-kernel geometry")
    M = N * T * H * W
    g = torch.Generator().manual_seed(ci + 3 * co + len(mode))
    spec = ConvSpec(ci, co, (1, 1, 1))
    w = torch.randn(co, ci, 1, 1, 1, generator=g) * (2.0 / ci) ** 0.5
    _, wd = pack_weight(w.to(DEV), spec)
    dy = torch.randn(M, co, generator=g).to(torch.bfloat16).to(DEV)
    bf = lambda *s: torch.randn(*s, generator=g).to(torch.bfloat16).to(DEV)
    res, old, y0, y1 = bf(M, ci), bf(M, ci), bf(M, ci) * 2 + 0.5, bf(M, ci)
    mask = torch.rand(M, ci, generator=g).to(DEV) > 0.4
    mean0, rstd0 = (torch.randn(ci, generator=g) * 0.3).to(DEV), (torch.rand(ci, generator=g) + 0.5).to(DEV)
    mean1, rstd1 = (torch.randn(ci, generator=g) * 0.3).to(DEV), (torch.rand(ci, generator=g) + 0.5).to(DEV)
    msc, msh = (torch.rand(ci, generator=g) + 0.2).to(DEV), (torch.randn(ci, generator=g) * 0.5).to(DEV)
    bias = (torch.randn(ci, generator=g) * 0.3).to(DEV)
    geo = dgrad_phases(spec, N, (T, H, W), (T, H, W), co, ci)
    assert len(geo) == 1 and C.conv_pw_legal(list(geo[0]), 8)
    dx = dy.double() @ w.view(co, ci).to(torch.bfloat16).double().to(DEV)
    for cfg in _cfgs():
        rows = C.conv_cfg_bm(cfg, ci)
        part = torch.full(((M + rows - 1) // rows, 3, ci), float("nan"), device=DEV)
        out = old.clone()
        if mode == "res_mask_dual_accum":
            C.conv_igemm_epi(dy, wd, out, 1, list(geo[0]), 8, res, ci, _bits(mask), y0, mean0, rstd0, y1, mean1,
                             rstd1, part, None, None, cfg)
            v = (dx + old.double() + res.double()) * mask
        elif mode == "bnmask_bias":
            C.conv_igemm_epi(dy, wd, out, 0, list(geo[0]), 8, None, 0, None, y0, mean0, rstd0, None, None, None,
                             part, msc, msh, cfg, bias)
            v = (dx + bias.double()) * ((y0.float() * msc + msh) > 0)
        else:
            C.conv_igemm_epi(dy, wd, out, 0, list(geo[0]), 8, None, 0, None, None, None, None, None, None, None,
                             part, None, None, cfg)
            v = dx
        torch.cuda.synchronize()
        assert _rel(out, v) < 1e-2, (cfg, mode)
        q = out.double()
        s = part.double().sum(0)
        assert _rel(s[0], q.sum(0)) < 1e-4, cfg
        if mode != "plain":
            ref1 = (q * (y0.double() - mean0.double()) * rstd0.double()).sum(0)
            assert (s[1] - ref1).abs().max().item() <= 1e-4 * (q.abs() * (y0.double() - mean0.double()).abs()
                                                                * rstd0.double()).sum(0).max().item(), cfg
        else:
            assert torch.all(s[1] == 0)
        if mode == "res_mask_dual_accum":
            ref2 = (q * (y1.double() - mean1.double()) * rstd1.double()).sum(0)
            assert (s[2] - ref2).abs().max().item() <= 1e-4 * (q.abs() * (y1.double() - mean1.double()).abs()
                                                                * rstd1.double()).sum(0).max().item(), cfg


def test_pw_legality():
    C = _C()
    spec3 = ConvSpec(64, 64, (1, 3, 3), (1, 1, 1), (0, 1, 1))
    assert not C.conv_pw_legal(list(fwd_geometry(spec3, 1, 2, 8, 8, 64, 64)), 8)
    s2 = ConvSpec(64, 256, (1, 1, 1), (1, 2, 2), (0, 0, 0))
    assert not C.conv_pw_legal(list(fwd_geometry(s2, 1, 2, 8, 8, 64, 256)), 8)
    big = ConvSpec(256, 1024, (1, 1, 1))   # 512 KB of weights: output-channel groups
    assert C.conv_pw_legal(list(fwd_geometry(big, 1, 2, 8, 8, 256, 1024)), 8)
    deep = ConvSpec(512, 256, (1, 1, 1))   # K > 256
    assert not C.conv_pw_legal(list(fwd_geometry(deep, 1, 2, 8, 8, 512, 256)), 8)
    n16 = ConvSpec(64, 16, (1, 1, 1))      # N % 32 != 0
    assert not C.conv_pw_legal(list(fwd_geometry(n16, 1, 2, 8, 8, 64, 16)), 8)
    ok = ConvSpec(64, 256, (1, 1, 1))
    assert C.conv_pw_legal(list(fwd_geometry(ok, 1, 2, 8, 8, 64, 256)), 8)


def _rows(t):   # [N, C, T, H, W] -> rows [N*T*H*W, C]
    return t.permute(0, 2, 3, 4, 1).reshape(-1, t.shape[1])


# temporal (kt,1,1) unit-stride convs on the pointwise kernel's temporal-tap loader: (N, T, H, W), Cin, Cout, kt
TEMPORAL = [((2, 4, 6, 7), 32, 32, 3), ((1, 8, 7, 7), 64, 64, 3), ((2, 3, 8, 8), 16, 32, 5), ((1, 5, 6, 6), 8, 96, 3),
            ((1, 4, 7, 9), 64, 128, 3)]


@pytest.mark.parametrize("case", TEMPORAL)
@pytest.mark.parametrize("aff", [0, 2])
def test_pw_temporal_forward(case, aff):
    """(kt,1,1) conv with temporal zero padding (taps leaving the clip read zero, also under the input BN-ReLU),
    accumulate + bias, forward BN partial sums, against PyTorch conv3d in float64."""
    C = _C()
    (N, T, H, W), ci, co, kt = case
    M = N * T * H * W
    g = torch.Generator().manual_seed(ci + co + kt + aff)
    spec = ConvSpec(ci, co, (kt, 1, 1), (1, 1, 1), (kt // 2, 0, 0))
    w = torch.randn(co, ci, kt, 1, 1, generator=g) * (2.0 / (ci * kt)) ** 0.5
    wf, _ = pack_weight(w.to(DEV), spec)
    x = torch.randn(M, ci, generator=g).to(torch.bfloat16).to(DEV)
    sc = (torch.rand(ci, generator=g) + 0.5).to(DEV)
    sh = (torch.randn(ci, generator=g) * 0.3).to(DEV)
    bias = (torch.randn(co, generator=g) * 0.2).to(DEV)
    xin = x.double() if not aff else torch.relu(x.float() * sc + sh).to(torch.bfloat16).double()
    xin = xin.view(N, T, H, W, ci).permute(0, 4, 1, 2, 3)
    ref0 = _rows(torch.nn.functional.conv3d(xin, w.to(torch.bfloat16).double().to(DEV), None, 1, (kt // 2, 0, 0)))
    geo = fwd_geometry(spec, N, T, H, W, ci, co)
    assert C.conv_pw_legal(list(geo), 8)
    for cfg in _cfgs():
        for accum, use_bias in ((0, False), (1, True)):
            y = torch.randn(M, co, generator=g).to(torch.bfloat16).to(DEV)
            old = y.clone()
            rows = C.conv_cfg_bm(cfg, co)
            stats = torch.full(((M + rows - 1) // rows, 2, co), float("nan"), device=DEV)
            C.conv_igemm(x, wf, y, stats, sc if aff else None, sh if aff else None, aff, accum, list(geo), 8, cfg,
                         bias if use_bias else None)
            torch.cuda.synchronize()
            ref = ref0 + (bias.double() if use_bias else 0) + (old.double() if accum else 0)
            assert _rel(y, ref) < 8e-3, (cfg, accum)
            q = y.double()
            s = stats.double().sum(0)
            assert _rel(s[0], q.sum(0)) < 1e-4 and _rel(s[1], (q * q).sum(0)) < 1e-4, cfg


# dgrad geometries the kernel takes: N = Cin % 32 == 0, K = kt x Cout <= 256
TEMPORAL_DGRAD = [((2, 4, 6, 7), 32, 32, 3), ((1, 8, 7, 7), 64, 64, 3), ((2, 4, 8, 8), 64, 32, 5),
                  ((1, 6, 6, 6), 128, 64, 3)]


@pytest.mark.parametrize("case", TEMPORAL_DGRAD)
@pytest.mark.parametrize("mode", ["res_mask_dual_accum", "plain"])
def test_pw_temporal_dgrad(case, mode):
    """dgrad of a (kt,1,1) stride-1 conv (taps gathered backwards) with the backward-BN epilogue, against
    torch.nn.grad.conv3d_input in float64."""
    C = _C()
    (N, T, H, W), ci, co, kt = case
    M = N * T * H * W
    g = torch.Generator().manual_seed(3 * ci + co + kt + len(mode))
    spec = ConvSpec(ci, co, (kt, 1, 1), (1, 1, 1), (kt // 2, 0, 0))
    w = torch.randn(co, ci, kt, 1, 1, generator=g) * (2.0 / (ci * kt)) ** 0.5
    _, wd = pack_weight(w.to(DEV), spec)
    dy = torch.randn(M, co, generator=g).to(torch.bfloat16).to(DEV)
    bf = lambda *s: torch.randn(*s, generator=g).to(torch.bfloat16).to(DEV)
    res, old, y0, y1 = bf(M, ci), bf(M, ci), bf(M, ci) * 2 + 0.5, bf(M, ci)
    mask = torch.rand(M, ci, generator=g).to(DEV) > 0.4
    mean0, rstd0 = (torch.randn(ci, generator=g) * 0.3).to(DEV), (torch.rand(ci, generator=g) + 0.5).to(DEV)
    mean1, rstd1 = (torch.randn(ci, generator=g) * 0.3).to(DEV), (torch.rand(ci, generator=g) + 0.5).to(DEV)
    geo = dgrad_phases(spec, N, (T, H, W), (T, H, W), co, ci)
    assert len(geo) == 1 and C.conv_pw_legal(list(geo[0]), 8)
    dyn = dy.double().view(N, T, H, W, co).permute(0, 4, 1, 2, 3)
    dx = _rows(torch.nn.grad.conv3d_input((N, ci, T, H, W), w.to(torch.bfloat16).double().to(DEV), dyn, 1,
                                          (kt // 2, 0, 0)))
    for cfg in _cfgs():
        rows = C.conv_cfg_bm(cfg, ci)
        part = torch.full(((M + rows - 1) // rows, 3, ci), float("nan"), device=DEV)
        out = old.clone()
        if mode == "res_mask_dual_accum":
            C.conv_igemm_epi(dy, wd, out, 1, list(geo[0]), 8, res, ci, _bits(mask), y0, mean0, rstd0, y1, mean1,
                             rstd1, part, None, None, cfg)
            v = (dx + old.double() + res.double()) * mask
        else:
            C.conv_igemm_epi(dy, wd, out, 0, list(geo[0]), 8, None, 0, None, None, None, None, None, None, None,
                             part, None, None, cfg)
            v = dx
        torch.cuda.synchronize()
        assert _rel(out, v) < 1e-2, (cfg, mode)
        assert _rel(part.double().sum(0)[0], out.double().sum(0)) < 1e-4, cfg


def test_pw_temporal_legality():
    C = _C()
    t3 = ConvSpec(32, 32, (3, 1, 1), (1, 1, 1), (1, 0, 0))
    assert C.conv_pw_legal(list(fwd_geometry(t3, 2, 4, 6, 7, 32, 32)), 8)
    assert C.conv_pw_legal(list(dgrad_phases(t3, 2, (4, 6, 7), (4, 6, 7), 32, 32)[0]), 8)
    assert not C.conv_pw_legal(list(fwd_geometry(t3, 2, 4, 5, 5, 32, 32)), 8)       # slices < 32 pixels
    deep = ConvSpec(128, 32, (3, 1, 1), (1, 1, 1), (1, 0, 0))                       # K = 384
    assert not C.conv_pw_legal(list(fwd_geometry(deep, 1, 4, 8, 8, 128, 32)), 8)
    st2 = ConvSpec(32, 32, (3, 1, 1), (2, 1, 1), (1, 0, 0))                         # temporal stride
    assert not C.conv_pw_legal(list(fwd_geometry(st2, 1, 4, 8, 8, 32, 32)), 8)
    sp = ConvSpec(32, 32, (1, 3, 3), (1, 1, 1), (0, 1, 1))                          # spatial taps
    assert not C.conv_pw_legal(list(fwd_geometry(sp, 1, 4, 8, 8, 32, 32)), 8)


@pytest.mark.parametrize("case", [FWD[0], FWD[2], FWD[6]])
def test_pw_statistics_only(case):
    """nostore (the narrow BN fold's exact-statistics pass): the same per-tile BN partial sums as a storing launch,
    and nothing written."""
    C = _C()
    (N, T, H, W), ci, co, _, _ = case
    M = N * T * H * W
    g = torch.Generator().manual_seed(ci + co)
    spec = ConvSpec(ci, co, (1, 1, 1))
    w = torch.randn(co, ci, 1, 1, 1, generator=g) * (2.0 / ci) ** 0.5
    wf, _ = pack_weight(w.to(DEV), spec)
    x = torch.randn(M, ci, generator=g).to(torch.bfloat16).to(DEV)
    sc = (torch.rand(ci, generator=g) + 0.5).to(DEV)
    sh = (torch.randn(ci, generator=g) * 0.3).to(DEV)
    geo = fwd_geometry(spec, N, T, H, W, ci, co)
    for cfg in _cfgs():
        rows = C.conv_cfg_bm(cfg, co)
        tiles = (M + rows - 1) // rows
        y = torch.empty(M, co, device=DEV, dtype=torch.bfloat16)
        ref = torch.full((tiles, 2, co), float("nan"), device=DEV)
        C.conv_igemm(x, wf, y, ref, sc, sh, 2, 0, list(geo), 8, cfg, None, 0)
        dummy = torch.zeros(1, 8, device=DEV, dtype=torch.bfloat16)
        got = torch.full((tiles, 2, co), float("nan"), device=DEV)
        C.conv_igemm(x, wf, dummy, got, sc, sh, 2, 0, list(geo), 8, cfg, None, 1)
        torch.cuda.synchronize()
        assert torch.equal(got, ref), cfg
        assert torch.all(dummy == 0)
