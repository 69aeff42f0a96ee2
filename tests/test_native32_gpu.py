"""fp32 path (csrc/fp32, models/native32.py) against plain PyTorch fp32/fp64 references.

* every convolution geometry family of SlowFast / Slow-R50 (stems with RGB padded to 4 channels, temporal conv_a,
  strided and stride-1 conv_b, strided 1x1 branch1, lateral (7,1,1)/(4,1,1), fast stem (5,7,7)): forward, stride-phase
  input gradient (plain and accumulating) and weight gradient vs an fp64 CPU oracle — three pieces (bf16x6, the
  default) < 2e-6 relative L2, two pieces (bf16x3) ~1e-5;
* the pre-split weight planes (three bf16 pieces summing to the fp32 weight);
* BatchNorm train forward (statistics, running-stat update) + backward, max pool and stride-1 average pool;
* whole networks (SlowFast-R50 and Slow-R50): one training step at small shapes against the PyTorch fp32 module path
  (median per-parameter gradient error within 3x of stock fp32's own distance to an fp64 run, or 1e-3), and at the
  full shapes against an fp64 oracle next to stock fp32 (median within 1.5x, worst within 2x of stock fp32's error):
  two correct fp32 executions of these random-init BN networks differ by ~2e-2 per parameter, so a fixed 1e-3 gate
  between them is not attainable (profiles/r6_f32/README.md);
* gradient accumulation into the flat buffer and the per-parameter progress hook.
"""
import pytest
import torch
import torch.nn.functional as Fnn

from pytorchvideo_accelerate_amd.ops._ext import require
from pytorchvideo_accelerate_amd.ops.f32 import ConvGeom, conv_dgrad, conv_fwd, conv_wgrad, pack_weight

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (cin, cout, k, s, p, N, T, H, W)
CONVS = [
    (3, 64, (1, 7, 7), (1, 2, 2), (0, 3, 3), 2, 2, 32, 32),     # slow stem (RGB padded to 4)
    (3, 8, (5, 7, 7), (1, 2, 2), (2, 3, 3), 1, 6, 24, 24),      # fast stem
    (64, 64, (1, 1, 1), (1, 1, 1), (0, 0, 0), 2, 2, 14, 14),    # 1x1
    (80, 64, (3, 1, 1), (1, 1, 1), (1, 0, 0), 2, 4, 14, 14),    # temporal conv_a on a lateral concat (80 ch)
    (64, 64, (1, 3, 3), (1, 1, 1), (0, 1, 1), 2, 2, 14, 14),    # conv_b
    (128, 128, (1, 3, 3), (1, 2, 2), (0, 1, 1), 1, 2, 14, 14),  # strided conv_b (4 phases)
    (256, 512, (1, 1, 1), (1, 2, 2), (0, 0, 0), 1, 2, 14, 14),  # strided branch1 (3 empty phases)
    (8, 16, (7, 1, 1), (4, 1, 1), (3, 0, 0), 2, 16, 8, 8),      # lateral fast->slow
    (8, 8, (3, 1, 1), (1, 1, 1), (1, 0, 0), 2, 8, 12, 12),      # narrow fast conv_a
    (2048, 256, (1, 1, 1), (1, 1, 1), (0, 0, 0), 1, 1, 7, 7),   # wide K, partial M tile
    (32, 2048, (1, 1, 1), (1, 1, 1), (0, 0, 0), 1, 2, 7, 7),    # wide N
]


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _ndhwc(x, cp=None):
    x = x.permute(0, 2, 3, 4, 1)
    if cp and cp > x.shape[-1]:
        x = torch.cat([x, torch.zeros(*x.shape[:-1], cp - x.shape[-1], dtype=x.dtype)], -1)
    return x.contiguous()


@pytest.mark.parametrize("pieces", [3, 2])
@pytest.mark.parametrize("case", CONVS)
def test_conv32_fwd_dgrad_wgrad(case, pieces, monkeypatch):
    """pieces 3 (default): fp32-class error (~1e-7 relative to the fp64 oracle); pieces 2: ~1e-5."""
    monkeypatch.setenv("PVA_ARMS", f"f32_pieces={pieces}")
    tol = 2e-6 if pieces == 3 else 3e-5
    cin, cout, k, s, p, N, T, H, W = case
    F = require().f32
    g = torch.Generator().manual_seed(11)
    x = torch.randn(N, cin, T, H, W, generator=g, dtype=torch.float64)
    w = torch.randn(cout, cin, *k, generator=g, dtype=torch.float64) / (cin * k[0] * k[1] * k[2]) ** 0.5
    x.requires_grad_(True)
    w.requires_grad_(True)
    y = Fnn.conv3d(x, w, None, s, p)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    y.backward(dy)
    geo = ConvGeom(cin, cout, k, s, p, cip=(cin + 3) // 4 * 4)
    xd = _ndhwc(x.detach(), geo.cip).float().to(DEV)
    wd = w.detach().float().to(DEV).contiguous()
    wf = pack_weight(F, geo, wd, 0)
    yd = torch.empty(N, *y.shape[2:], cout, device=DEV)
    M = yd.numel() // cout
    st = torch.full((-(-M // F.igemm32_bm(cout)), 2, cout), float("nan"), device=DEV)
    conv_fwd(F, geo, xd, wf, yd, geo.taps_fwd(DEV), stats=st)
    assert _rel(yd, _ndhwc(y.detach())) < tol
    # epilogue BatchNorm statistics: per-tile sums of y and y^2 (every tile row written)
    y2 = yd.reshape(M, cout).double()
    assert torch.isfinite(st).all()
    assert _rel(st[:, 0].double().sum(0), y2.sum(0)) < 1e-5 and _rel(st[:, 1].double().sum(0), (y2 * y2).sum(0)) < 1e-5
    dyd = _ndhwc(dy).float().to(DEV)
    # weight gradient
    dwf = torch.empty(cout, geo.ntap * geo.cip, device=DEV)
    F.zero32(dwf)
    conv_wgrad(F, geo, dyd, xd, dwf, geo.taps_fwd(DEV))
    dw = torch.full_like(wd, 7.0)
    F.wpack32(2, dwf, dw, cout, cin, geo.ntap, geo.cip, 0.0)
    assert _rel(dw, w.grad) < tol
    # accumulate form (beta = 1)
    dw2 = dw.clone()
    F.wpack32(2, dwf, dw2, cout, cin, geo.ntap, geo.cip, 1.0)
    assert _rel(dw2, 2 * w.grad) < tol
    if cin % 4:
        return
    wt = pack_weight(F, geo, wd, 1)
    dx = torch.full((N, T, H, W, cin), float("nan"), device=DEV)   # every position must be written
    conv_dgrad(F, geo, dyd, wt, dx, geo.phases(DEV))
    assert torch.isfinite(dx).all()
    assert _rel(dx, _ndhwc(x.grad)) < tol


def test_pack_weight_planes():
    """wpack32 modes 0 / 1: three bf16 pieces whose sum is the fp32 weight (24 significant bits) in the forward
    ([Cout][taps][cip], padded channels zero) and input-gradient ([Cin][taps][Cout]) row layouts."""
    F = require().f32
    g = ConvGeom(3, 8, (3, 3, 3), (1, 1, 1), (1, 1, 1), cip=4)
    w = torch.randn(8, 3, 3, 3, 3, device=DEV) * 1e-2
    wf = pack_weight(F, g, w, 0)
    assert wf.shape == (3, 8, 27 * 4) and wf.dtype == torch.bfloat16
    ref = torch.zeros(8, 27, 4, device=DEV, dtype=torch.float64)
    ref[:, :, :3] = w.double().reshape(8, 3, 27).permute(0, 2, 1)
    got = wf.double().sum(0).reshape(8, 27, 4)
    assert (got - ref).abs().max() <= 2 ** -24 * ref.abs().max()
    g2 = ConvGeom(4, 8, (1, 3, 3), (1, 1, 1), (0, 1, 1))
    w2 = torch.randn(8, 4, 1, 3, 3, device=DEV)
    wt = pack_weight(F, g2, w2, 1)
    ref2 = w2.double().reshape(8, 4, 9).permute(1, 2, 0)
    assert wt.shape == (3, 4, 9 * 8)
    assert (wt.double().sum(0).reshape(4, 9, 8) - ref2).abs().max() <= 2 ** -24 * ref2.abs().max()


def test_dgrad_accumulate_phases():
    """The executor's accumulating input gradient (residual / lateral sums) on a strided conv."""
    from pytorchvideo_accelerate_amd.models.native32 import _ConvBN
    F = require().f32
    torch.manual_seed(0)
    conv = torch.nn.Conv3d(64, 128, (1, 3, 3), (1, 2, 2), (0, 1, 1), bias=False).to(DEV)
    bn = torch.nn.BatchNorm3d(128).to(DEV)

    class _N:
        device = torch.device(DEV)
    n = _N()
    n.F = F
    cb = _ConvBN(n, conv, bn, True)
    dy = torch.randn(2, 2, 7, 7, 128, device=DEV)
    wt = pack_weight(F, cb.g, conv.weight.detach(), 1)
    base = torch.randn(2, 2, 14, 14, 64, device=DEV)
    acc = base.clone()
    cb._dgrad(dy, wt, acc, True)
    ref = torch.nn.grad.conv3d_input((2, 64, 2, 14, 14), conv.weight.detach().double(),
                                     dy.permute(0, 4, 1, 2, 3).double(), (1, 2, 2), (0, 1, 1))
    assert _rel(acc - base, _ndhwc(ref)) < 2e-6


@pytest.mark.parametrize("C,M,relu,add", [(64, 3000, True, False), (8, 50000, True, True), (2048, 98, False, True),
                                          (80, 1000, True, False)])
def test_bn32_train_forward_backward(C, M, relu, add):
    F = require().f32
    torch.manual_seed(1)
    y = (torch.randn(M, C, dtype=torch.float64) * 3 + 1.5)
    gamma = torch.rand(C, dtype=torch.float64) + 0.5
    beta = torch.randn(C, dtype=torch.float64)
    a = torch.randn(M, C, dtype=torch.float64) if add else None
    yr = y.clone().requires_grad_(True)
    gr = gamma.clone().requires_grad_(True)
    br = beta.clone().requires_grad_(True)
    ar = a.clone().requires_grad_(True) if add else None
    mean = yr.mean(0)
    var = yr.var(0, unbiased=False)
    o = (yr - mean) / torch.sqrt(var + 1e-5) * gr + br
    if add:
        o = o + ar
    if relu:
        o = torch.relu(o)
    dout = torch.randn(M, C, dtype=torch.float64)
    o.backward(dout)
    yd, gd, bd = y.float().to(DEV), gamma.float().to(DEV), beta.float().to(DEV)
    rm = torch.zeros(C, device=DEV)
    rv = torch.ones(C, device=DEV)
    nbt = torch.zeros((), dtype=torch.long, device=DEV)
    part = torch.empty(F.chan_reduce32_blocks(M, C), 2, C, device=DEV)
    F.chan_reduce32(yd, C, None, C, None, C, None, 0, 0, M, C, part)
    stat = torch.empty(4, C, device=DEV)
    F.bn32_finalize(part, C, M, 0, gd, bd, rm, rv, nbt, 0.1, 1e-5, stat, None, None, None, None, 0.0)
    out = torch.empty(M, C, device=DEV)
    ad = a.float().to(DEV) if add else None
    F.bn32_apply(yd, C, stat, ad, C, int(relu), out, C, M, C)
    assert _rel(out, o.detach()) < 1e-5
    assert _rel(rm, 0.1 * y.mean(0)) < 1e-5
    assert _rel(rv, 0.9 + 0.1 * y.var(0, unbiased=True)) < 1e-5
    assert int(nbt) == 1
    dd = dout.float().to(DEV)
    part2 = torch.empty_like(part)
    F.chan_reduce32(yd, C, dd, C, out if relu else None, C, stat[0], 1, int(relu), M, C, part2)
    coef = torch.empty(3, C, device=DEV)
    dg = torch.full((C,), 100.0, device=DEV)
    db = torch.full((C,), 100.0, device=DEV)
    F.bn32_finalize(part2, C, M, 1, gd, bd, None, None, None, 0.0, 1e-5, None, stat, dg, db, coef, 1.0)
    dyd = torch.empty(M, C, device=DEV)
    gout = torch.empty(M, C, device=DEV)
    F.bn32_bwd_apply(dd, C, out if relu else None, C, int(relu), yd, C, stat, coef, dyd, C, gout, C, M, C)
    assert _rel(dyd, yr.grad) < 1e-4
    if relu and not add:   # the lazy-activation form: no stored output, the ReLU mask recomputed from y and stat
        part3 = torch.empty_like(part)
        F.chan_reduce32(yd, C, dd, C, None, C, stat[0], 1, 1, M, C, part3)
        assert torch.equal(part3, part2)
        dy3 = torch.empty(M, C, device=DEV)
        F.bn32_bwd_apply(dd, C, None, C, 1, yd, C, stat, coef, dy3, C, None, C, M, C)
        assert torch.equal(dy3, dyd)
    assert _rel(dg - 100.0, gr.grad) < 1e-4
    assert _rel(db - 100.0, br.grad) < 1e-4
    if add:
        assert _rel(gout, ar.grad) < 1e-6


def test_maxpool32_and_avgpool32():
    F = require().f32
    torch.manual_seed(2)
    N, C, T, H, W = 2, 8, 3, 17, 16
    x = torch.randn(N, C, T, H, W, dtype=torch.float64, requires_grad=True)
    y = Fnn.max_pool3d(x, (1, 3, 3), (1, 2, 2), (0, 1, 1))
    dy = torch.randn(y.shape, dtype=torch.float64)
    y.backward(dy)
    To, Ho, Wo = y.shape[2:]
    xd = _ndhwc(x.detach()).float().to(DEV)
    out = torch.empty(N, To, Ho, Wo, C, device=DEV)
    arg = torch.empty(N, To, Ho, Wo, C, device=DEV, dtype=torch.uint8)
    F.maxpool32(0, xd, out, arg, [N, T, H, W, To, Ho, Wo, C], [1, 3, 3], [1, 2, 2], [0, 1, 1])
    assert _rel(out, _ndhwc(y.detach())) < 1e-7
    dx = torch.empty_like(xd)
    F.maxpool32(1, _ndhwc(dy).float().to(DEV), dx, arg, [N, T, H, W, To, Ho, Wo, C], [1, 3, 3], [1, 2, 2], [0, 1, 1])
    assert _rel(dx, _ndhwc(x.grad)) < 1e-6
    # stride-1 average pool into a channel slice of the head features, and its backward
    x2 = torch.randn(N, C, 4, 8, 8, dtype=torch.float64, requires_grad=True)
    k = (4, 7, 7)
    p2 = Fnn.avg_pool3d(x2, k, 1)                     # [N, C, 1, 2, 2]
    P = p2.shape[2] * p2.shape[3] * p2.shape[4]
    dp = torch.randn(p2.shape, dtype=torch.float64)
    p2.backward(dp)
    Ct, coff = C + 4, 4
    feat = torch.zeros(N, P, Ct, device=DEV)
    F.avgpool32(0, _ndhwc(x2.detach()).float().to(DEV), feat, [N, 4, 8, 8, C], list(k), Ct, coff)
    ref = p2.detach().reshape(N, C, P).transpose(1, 2)
    assert _rel(feat[..., coff:], ref) < 1e-6
    dfeat = torch.zeros(N, P, Ct, device=DEV)
    dfeat[..., coff:] = dp.reshape(N, C, P).transpose(1, 2).float().to(DEV)
    dx2 = torch.empty(N, 4, 8, 8, C, device=DEV)
    F.avgpool32(1, dfeat, dx2, [N, 4, 8, 8, C], list(k), Ct, coff)
    assert _rel(dx2, _ndhwc(x2.grad)) < 1e-6


def _prel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _net_case(slowfast: bool):
    from pytorchvideo_accelerate_amd.models import reference as R
    torch.manual_seed(5)
    if slowfast:
        T, S = 16, 64
        model = R.create_slowfast(50, 11, head_pool_kernel_sizes=((T // 4, 2, 2), (T, 2, 2)), dropout_rate=0.0)
        fast = torch.randn(2, 3, T, S, S)
        xs = [fast[:, :, ::4].contiguous(), fast]
    else:
        T, S = 8, 64
        model = R.create_resnet(50, 11, head_pool_kernel_size=(T, 2, 2), dropout_rate=0.0)
        xs = torch.randn(2, 3, T, S, S)
    labels = torch.tensor([3, 7])
    return model, xs, labels


@pytest.mark.parametrize("slowfast", [True, False], ids=["slowfast_r50", "slow_r50"])
def test_native32_net_matches_torch_fp32(slowfast):
    """One training step against an fp64 oracle (the same module tree in float64 on the CPU).  The stock PyTorch fp32
    GPU step (MIOpen) is measured against the same oracle as the fp32 noise floor: a 50-layer train-mode BN network at
    B=2 amplifies per-op rounding (stock fp32 itself lands ~1e-2 from fp64 in gradient rel-L2 here), so agreement is
    judged relative to that floor: logits and the median / worst per-parameter gradient error within 3x of stock
    fp32's (round 6 measured bf16x3 pieces at 7-10x: the reason the default is three pieces)."""
    import copy
    from pytorchvideo_accelerate_amd.models.native32 import NativeF32Net
    model, xs, labels = _net_case(slowfast)
    ref64 = copy.deepcopy(model).double().train()
    x64 = [x.double() for x in xs] if isinstance(xs, list) else xs.double()
    out64 = ref64(x64)
    loss64 = Fnn.cross_entropy(out64, labels)
    loss64.backward()
    ref32 = copy.deepcopy(model).to(DEV).train()
    xin = [x.to(DEV) for x in xs] if isinstance(xs, list) else xs.to(DEV)
    out32 = ref32(xin)
    Fnn.cross_entropy(out32, labels.to(DEV)).backward()
    net = NativeF32Net(model, DEV)
    net.model.train()
    loss, logits = net.forward_backward(xs, labels, 1.0)
    torch.cuda.synchronize()
    g64 = dict(ref64.named_parameters())
    g32 = dict(ref32.named_parameters())
    ours, stock = {}, {}
    for n, p in model.named_parameters():
        ours[n] = _prel(net.flat.gview(p), g64[n].grad)
        stock[n] = _prel(g32[n].grad, g64[n].grad)
    med = lambda d: sorted(d.values())[len(d) // 2]   # noqa: E731
    worst = max(ours, key=ours.get)
    for n in list(ours)[:6] + [worst]:
        print(f"  {n}: ours {ours[n]:.2e} stock {stock[n]:.2e}")
    print(f"\nlogits rel: ours {_prel(logits, out64):.2e} stock-fp32 {_prel(out32, out64):.2e}; loss {loss.item():.6f} "
          f"vs {loss64.item():.6f}; grad rel-L2 median ours {med(ours):.2e} stock {med(stock):.2e}; worst ours "
          f"{ours[worst]:.2e} ({worst}) stock {max(stock.values()):.2e}")
    assert abs(loss.item() - loss64.item()) < 1e-4 * max(1.0, abs(loss64.item()))
    assert _prel(logits, out64) < max(1e-5, 3 * _prel(out32, out64))
    assert med(ours) < max(1e-3, 3 * med(stock))
    assert ours[worst] < max(1e-2, 3 * max(stock.values())), (worst, ours[worst])
    for (n, b), (_, b64) in zip(model.named_buffers(), ref64.named_buffers()):
        if b.dtype.is_floating_point:
            assert _prel(b, b64) < 1e-4, n
        else:
            assert int(b) == int(b64), n
    # eval forward (running statistics) matches the module path too
    ref64.eval()
    net.model.eval()
    with torch.no_grad():
        e64 = ref64(x64)
    e = net.forward_eval(xs)
    assert _prel(e, e64) < 1e-4


@pytest.mark.parametrize("arch", ["slowfast_r50", "slow_r50"])
def test_native32_full_shape_vs_fp64(arch):
    """Full-shape training step (SlowFast-R50 32x2x224; Slow-R50 8x8x224, the reference default model, run.py:338-351)
    against an fp64 oracle of the same module tree on the GPU, with the stock PyTorch fp32 step (MIOpen) judged
    against the same oracle as the fp32 floor.  Two correct fp32 executions of this network disagree in gradient
    rel-L2 by ~1e-2 (BN + ReLU amplify rounding; round 6: the native fp32 executor vs stock fp32 at B=4 had median
    2.6e-2 while the loss agreed to 3e-7), so the gates are relative to stock fp32's own error: median and worst
    per-parameter gradient error at most 1.5x / 2x stock's, logits and loss at fp32 level."""
    import copy
    from pytorchvideo_accelerate_amd.models import reference as R
    from pytorchvideo_accelerate_amd.models.native32 import NativeF32Net
    torch.manual_seed(3)
    g = torch.Generator().manual_seed(4)
    B = 2
    if arch == "slowfast_r50":
        model = R.create_slowfast(50, 400, dropout_rate=0.0)
        fast = torch.randn(B, 3, 32, 224, 224, generator=g)
        xs = [fast[:, :, torch.linspace(0, 31, 8).long()].contiguous(), fast]
    else:
        model = R.create_resnet(50, 400, head_pool_kernel_size=(8, 7, 7), dropout_rate=0.0)
        xs = torch.randn(B, 3, 8, 224, 224, generator=g)
    labels = torch.randint(0, 400, (B,), generator=g)

    def torch_step(dtype):
        m = copy.deepcopy(model).to(DEV, dtype).train()
        xin = [x.to(DEV, dtype) for x in xs] if isinstance(xs, list) else xs.to(DEV, dtype)
        out = m(xin)
        loss = Fnn.cross_entropy(out, labels.to(DEV))
        loss.backward()
        return m, out.detach(), loss.item()

    m64, out64, loss64 = torch_step(torch.float64)
    m32, out32, loss32 = torch_step(torch.float32)
    net = NativeF32Net(model, DEV)
    loss, logits = net.forward_backward(xs, labels, 1.0)
    torch.cuda.synchronize()
    g64, g32 = dict(m64.named_parameters()), dict(m32.named_parameters())
    ours = {n: _prel(net.flat.gview(p), g64[n].grad) for n, p in model.named_parameters()}
    stock = {n: _prel(g32[n].grad, g64[n].grad) for n in ours}
    vs_stock = {n: _prel(net.flat.gview(p), g32[n].grad) for n, p in model.named_parameters()}
    med = lambda d: sorted(d.values())[len(d) // 2]   # noqa: E731
    print(f"\n{arch}: loss ours {loss.item():.7f} stock {loss32:.7f} fp64 {loss64:.7f}; logits rel ours "
          f"{_prel(logits, out64):.2e} stock {_prel(out32, out64):.2e}; grad rel-L2 vs fp64 median ours {med(ours):.2e} "
          f"stock {med(stock):.2e}, worst ours {max(ours.values()):.2e} stock {max(stock.values()):.2e}; ours vs "
          f"stock median {med(vs_stock):.2e}")
    assert abs(loss.item() - loss64) <= 2 * abs(loss32 - loss64) + 1e-6 * abs(loss64)
    assert _prel(logits, out64) <= 2 * _prel(out32, out64) + 1e-6
    assert med(ours) <= 1.5 * med(stock) + 1e-4
    assert max(ours.values()) <= 2 * max(stock.values()) + 1e-4


def test_native32_grad_accumulates_and_progress_hook():
    """Second micro-step adds into the flat gradient; the progress hook sees monotone offsets ending at the end."""
    from pytorchvideo_accelerate_amd.models.native32 import NativeF32Net
    model, xs, labels = _net_case(False)
    net = NativeF32Net(model, DEV)
    seen = []
    net.grad_hook = seen.append
    net.forward_backward(xs, labels, 1.0, accumulate=False)
    g1 = net.flat.grad.clone()
    assert seen == sorted(seen) and seen[-1] == net.flat.span(net.flat.params[-1])[1]
    # BN running statistics moved: undo by re-running at the same weights gives the same gradients (batch stats)
    net.forward_backward(xs, labels, 1.0, accumulate=True)
    assert _prel(net.flat.grad, 2 * g1) < 1e-5
