"""Fused lateral-connection backward (csrc/kernels/lateral_bwd.hip) against fp32 PyTorch references of the same op:
the BN-backward apply (ReLU mask from the forward affine) and the strided temporal input gradient of the fast->slow
conv (7,1,1) / stride (4,1,1) / pad 3, accumulated onto an existing gradient; channel-slice input (a concat view) and
padded output rows; partial position tiles and several 32-channel groups.  Then the whole executor with the fused path
against the unfused one (deterministic mode: identical loss, gradients within bf16 re-association noise)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _C():
    from pytorchvideo_accelerate_amd.ops._ext import require
    return require()


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("N,To,H,W,CO,Cf", [(2, 3, 5, 7, 64, 32), (1, 8, 10, 20, 128, 64), (3, 2, 16, 16, 64, 32),
                                            (2, 4, 9, 15, 16, 8), (1, 3, 14, 14, 256, 128)])
def test_lateral_bwd_matches_reference(N, To, H, W, CO, Cf):
    C = _C()
    torch.manual_seed(0)
    Tf, HW = 4 * To, H * W
    Ms, Mf = N * To * HW, N * Tf * HW
    bf = torch.bfloat16
    cat = torch.randn(Ms, CO + 40, device=DEV).to(bf)          # g: the last CO channels of a concat buffer
    g = cat[:, 40:]
    y = torch.randn(Ms, CO, device=DEV).to(bf)
    sc = torch.rand(CO, device=DEV) + 0.5
    sh = torch.randn(CO, device=DEV) * 0.5
    coef = torch.randn(3 * CO, device=DEV)
    Wt = (torch.randn(CO, Cf, 7, 1, 1, device=DEV) * 0.1).to(bf).float()
    wd = Wt.reshape(CO, Cf, 7).permute(1, 2, 0).contiguous().to(bf)   # dgrad pack [Cf][7][CO]
    ldx = Cf + 8
    dx = torch.randn(Mf, ldx, device=DEV).to(bf)
    old = dx.clone()
    dy = torch.empty(Ms, CO, device=DEV, dtype=bf)
    C.lateral_bwd(g, g.stride(0), y, sc, sh, coef, wd, dy, dx, ldx, N, To, Tf, HW, CO, Cf, 4)
    torch.cuda.synchronize()
    # apply
    yf, gf = y.float(), g.float()
    dz = torch.where(yf * sc + sh > 0, gf, torch.zeros_like(gf))
    dy_ref = coef[:CO] * dz + coef[CO:2 * CO] * yf + coef[2 * CO:]
    assert _rel(dy.float(), dy_ref) < 4e-3
    assert (dy.float() - dy_ref).abs().max().item() <= 2e-2 * dy_ref.abs().max().item()
    # dgrad of the kernel's own dy (isolates the strided accumulation), onto the old gradient
    dy5 = dy.float().view(N, To, H, W, CO).permute(0, 4, 1, 2, 3)
    dxi = torch.nn.grad.conv3d_input((N, Cf, Tf, H, W), Wt, dy5, stride=(4, 1, 1), padding=(3, 0, 0))
    ref = old[:, :Cf].float() + dxi.permute(0, 2, 3, 4, 1).reshape(Mf, Cf)
    assert _rel(dx[:, :Cf].float(), ref) < 4e-3, _rel(dx[:, :Cf].float(), ref)
    assert torch.equal(dx[:, Cf:], old[:, Cf:]), "padding columns of dx were written"
    # every frame was written exactly once: no frame kept its old value where the reference changed it
    moved = (ref - old[:, :Cf].float()).abs().view(N, Tf, HW, Cf).amax(dim=(0, 2, 3))
    got = (dx[:, :Cf].float() - old[:, :Cf].float()).abs().view(N, Tf, HW, Cf).amax(dim=(0, 2, 3))
    assert bool(((moved > 0) <= (got > 0)).all())


def test_lateral_fused_net_matches_unfused(monkeypatch):
    from pytorchvideo_accelerate_amd.models import reference as R
    from pytorchvideo_accelerate_amd.models.fused import FusedNet
    torch.manual_seed(0)
    model = R.create_slowfast(50, 10, head_pool_kernel_sizes=((2, 2, 2), (8, 2, 2)), dropout_rate=0.0)
    gen = torch.Generator().manual_seed(1)
    fast = torch.randn(2, 3, 8, 64, 64, generator=gen).to(torch.bfloat16).float()
    xs = [fast[:, :, torch.linspace(0, 7, 2).long()].contiguous(), fast]
    labels = torch.tensor([1, 7], device=DEV)
    runs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("PVA_ARMS", f"lateral_bwd={flag}")
        m = copy.deepcopy(model)
        eng = FusedNet(m, DEV, deterministic=True)
        loss, _ = eng.forward_backward(eng.prepare_inputs(xs), labels)
        torch.cuda.synchronize()
        fuses = [f for _, f in eng.stages if f is not None]
        runs.append((float(loss), {n: p.grad.detach().clone() for n, p in m.named_parameters()},
                     sum(f.lateral_used for f in fuses)))
    (l1, g1, n1), (l0, g0, n0) = runs
    assert n1 == 4 and n0 == 0, (n1, n0)   # the stem, res2, res3 and res4 laterals
    assert abs(l1 - l0) < 1e-6 * max(1.0, abs(l0)), (l1, l0)
    errs = sorted((_rel(g1[n], g0[n]), n) for n in g0 if g0[n].norm() > 0)
    # four re-associated kernels upstream of the fast stem: a BN bias gradient (a near-cancelling sum over 16M
    # positions) moves by a few %; the bulk stays at bf16 noise
    assert errs[len(errs) // 2][0] < 5e-3 and errs[-1][0] < 5e-2, (errs[len(errs) // 2], errs[-3:])
