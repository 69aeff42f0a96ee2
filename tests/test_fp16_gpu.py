"""fp16 compute (``--mixed_precision fp16``, the reference recipe run_slowfast_r50.sh:9 / run.py:135-136): the fp16
build of every kernel (csrc/kernels/common.h, namespace pva_f16, v_mfma_f32_16x16x32_f16) against plain PyTorch fp32
references of the same op, every launch configuration the autotuner can pick; the fused executor in fp16 against the
fp32 oracle within twice the fp16-autocast noise floor; and a fixed-batch fp16 training run with loss scaling whose
overflow back-off is exercised."""
import copy
import math

import pytest
import torch
import torch.nn.functional as F

from pytorchvideo_accelerate_amd.models import reference as R
from pytorchvideo_accelerate_amd.models.fused import FusedNet
from pytorchvideo_accelerate_amd.ops._ext import require
from pytorchvideo_accelerate_amd.ops.conv import (Act, ConvSpec, conv_dgrad, conv_wgrad, dgrad_phases, fwd_geometry,
                                                  pack_weight)
from pytorchvideo_accelerate_amd.ops.optim import FusedGradScaler, FusedSGD
from pytorchvideo_accelerate_amd.ops.tune import ConvTuner, describe

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
H = torch.float16

CASES = [
    (64, 256, (1, 1, 1), (1, 1, 1), (0, 0, 0), (2, 4, 14, 14)),      # slow pointwise (pw kernel)
    (256, 64, (3, 1, 1), (1, 1, 1), (1, 0, 0), (2, 8, 14, 14)),      # slow temporal
    (64, 64, (1, 3, 3), (1, 1, 1), (0, 1, 1), (2, 4, 14, 14)),       # slow spatial (halo kernels)
    (128, 128, (1, 3, 3), (1, 2, 2), (0, 1, 1), (2, 4, 28, 28)),     # spatial stride 2
    (8, 16, (7, 1, 1), (4, 1, 1), (3, 0, 0), (2, 32, 14, 14)),       # lateral fusion
    (8, 8, (1, 3, 3), (1, 1, 1), (0, 1, 1), (2, 16, 20, 20)),        # fast conv_b (narrow halo / direct)
    (32, 8, (3, 1, 1), (1, 1, 1), (1, 0, 0), (2, 16, 16, 16)),       # fast conv_a
    (512, 2048, (1, 1, 1), (1, 1, 1), (0, 0, 0), (2, 2, 7, 7)),      # res5 conv_c (256x256 tile)
]


def rel_err(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6)).item()


def _mk(case, seed=0):
    cin, cout, k, s, p, (N, T, Hh, W) = case
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, cin, T, Hh, W, generator=g).to(DEV).to(H).float()
    w = (torch.randn(cout, cin, *k, generator=g) / (cin * k[0] * k[1] * k[2]) ** 0.5).to(DEV).to(H).float()
    return x, w, ConvSpec(cin, cout, k, s, p)


@pytest.mark.parametrize("case", CASES)
def test_fp16_conv_fwd_every_config(case):
    """Forward (+ consumer-side BN-ReLU affine) of every legal launch configuration, fp16 operands vs fp32."""
    C = require()
    x, w, spec = _mk(case)
    sc = torch.rand(spec.cin, device=DEV) + 0.5
    sh = torch.randn(spec.cin, device=DEV) * 0.5
    xt = torch.relu(x * sc.view(1, -1, 1, 1, 1) + sh.view(1, -1, 1, 1, 1))
    ref = F.conv3d(xt, w, None, spec.stride, spec.pad)
    wf, _ = pack_weight(w, spec, H)
    xa = Act.from_ncthw(x, dtype=H)
    To, Ho, Wo = spec.out_dims(xa.T, xa.H, xa.W)
    M = xa.N * To * Ho * Wo
    g = fwd_geometry(spec, xa.N, xa.T, xa.H, xa.W, xa.ld, spec.cout)
    cands = ConvTuner(C).candidates(g, spec.chunk, aff=2)
    assert cands
    for cfg in [-1] + cands:
        y = torch.full((M, spec.cout), float("nan"), device=DEV, dtype=H)
        stats = torch.zeros((M + 15) // 16, 2, spec.cout, device=DEV)
        C.conv_igemm(xa.t, wf, y, stats, sc, sh, 2, 0, g, spec.chunk, cfg)
        out = y.view(xa.N, To, Ho, Wo, spec.cout).permute(0, 4, 1, 2, 3)
        assert y.dtype == H and rel_err(out, ref) < 1e-2, describe(cfg)
        yf = y.float()
        torch.testing.assert_close(stats.sum(0)[1], (yf * yf).sum(0), rtol=2e-3, atol=1e-2)


@pytest.mark.parametrize("case", [c for c in CASES if c[0] % 8 == 0])
def test_fp16_conv_dgrad_and_wgrad(case):
    C = require()
    x, w, spec = _mk(case, seed=1)
    gy = torch.randn(F.conv3d(x, w, None, spec.stride, spec.pad).shape, generator=torch.Generator().manual_seed(2))
    gy = gy.to(DEV).to(H).float()
    dx_ref = torch.nn.grad.conv3d_input(x.shape, w, gy, spec.stride, spec.pad)
    dw_ref = torch.nn.grad.conv3d_weight(x, w.shape, gy, spec.stride, spec.pad)
    _, wd = pack_weight(w, spec, H)
    dy = Act.from_ncthw(gy, dtype=H)
    dx = conv_dgrad(dy, wd, spec, tuple(x.shape[2:]))
    assert dx.t.dtype == H and rel_err(dx.to_ncthw(), dx_ref) < 1e-2
    # every dgrad launch configuration of the first phase
    g = dgrad_phases(spec, dy.N, tuple(x.shape[2:]), (dy.T, dy.H, dy.W), dy.ld, spec.cin)
    if len(g) == 1:
        for cfg in ConvTuner(C).candidates(g[0], 8):
            out = torch.full_like(dx.t, float("nan"))
            C.conv_igemm(dy.t, wd, out, None, None, None, 0, 0, g[0], 8, cfg)
            assert rel_err(out.view(dx.t.shape), dx.t.float()) < 1e-2, describe(cfg)
    xa = Act.from_ncthw(x, dtype=H)
    grad = torch.zeros_like(w)
    conv_wgrad(dy, xa, spec, grad)
    assert rel_err(grad, dw_ref) < 1e-2


def test_fp16_preprocess_matches_reference_transform():
    from pytorchvideo_accelerate_amd.data.transforms import GpuClipBatch, reference_transform, sample_params
    g = torch.Generator().manual_seed(5)
    B, Ts, Hs, Ws, T, S = 2, 24, 64, 80, 8, 48
    frames = torch.randint(0, 256, (B, Ts, Hs, Ws, 3), generator=g, dtype=torch.uint8)
    params = [sample_params(Ts, Hs, Ws, T, S, True, min_scale=52, max_scale=60, generator=g) for _ in range(B)]
    out = GpuClipBatch(DEV, T, S, None, dtype=H)(frames.to(DEV), params)[0]
    assert out.t.dtype == H
    for b in range(B):
        ref = reference_transform(frames[b], params[b], S)
        got = out.to_ncthw()[b, :3].float().cpu()
        # within one fp16 ulp (10 explicit significand bits) of the fp32 reference at every element; next to zero the
        # fp32 cancellation in x/255 - mean costs ~1e-7 absolute in both computations (floor 1e-6)
        ulp = torch.pow(2.0, torch.floor(torch.log2(ref.abs().clamp_min(2.0 ** -30))) - 10).clamp_min(1e-6)
        err = (got - ref).abs()
        assert (err <= ulp).all(), (float((err / ulp).max()), float(ref.flatten()[(err / ulp).argmax()]))


def _sf(classes=10):
    torch.manual_seed(0)
    return R.create_slowfast(50, classes, head_pool_kernel_sizes=((2, 2, 2), (8, 2, 2)), dropout_rate=0.0)


def _inputs(N=2, T=8, S=64, alpha=4, seed=0):
    g = torch.Generator().manual_seed(seed)
    fast = torch.randn(N, 3, T, S, S, generator=g).to(H).float()
    idx = torch.linspace(0, T - 1, T // alpha).long()
    return [fast[:, :, idx].contiguous(), fast]


def _grad_errs(model, oracle, ac):
    ref, acp = dict(oracle.named_parameters()), dict(ac.named_parameters())
    fe, ae = [], []
    for n, p in model.named_parameters():
        d = ref[n].grad.float().norm().clamp_min(1e-12)
        fe.append(((p.grad.float() - ref[n].grad.float()).norm() / d).item())
        ae.append(((acp[n].grad.float() - ref[n].grad.float()).norm() / d).item())
    return sorted(fe), sorted(ae)


@pytest.mark.parametrize("S,T,N", [(64, 8, 2), (224, 32, 2)])
def test_fp16_step_vs_fp32_oracle_within_autocast_noise(S, T, N):
    """One fused fp16 training step vs the fp32 oracle, judged against stock fp16 autocast of the same oracle: loss and
    per-parameter gradient rel-L2 (median and 90th percentile) within 2x the autocast noise floor.  Each side starts at
    GradScaler's 2^16 and halves the scale until its gradients are finite (the scaler's back-off, one skipped step
    per halving) — at 224^2 the stem's fp16 dgrad can overflow at 2^16 on randn input."""
    model = _sf() if S == 64 else R.create_slowfast(50, 400, dropout_rate=0.0)
    init = copy.deepcopy(model)
    xs = _inputs(N, T, S, seed=3)
    labels = torch.tensor([1, 7], device=DEV)
    oracle = copy.deepcopy(init).to(DEV).train()
    loss_ref = F.cross_entropy(oracle([x.to(DEV) for x in xs]), labels)
    loss_ref.backward()
    ac = copy.deepcopy(init).to(DEV).train()
    scale = 2.0 ** 16
    while True:
        ac.load_state_dict(init.state_dict())
        ac.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.float16):
            out_ac = ac([x.to(DEV) for x in xs])
        (F.cross_entropy(out_ac.float(), labels) * scale).backward()
        if all(torch.isfinite(p.grad).all() for p in ac.parameters()):
            break
        scale /= 2
    for p in ac.parameters():
        p.grad.div_(scale)
    loss_ac = F.cross_entropy(out_ac.float(), labels)
    eng = FusedNet(model, DEV, compute_dtype=H)
    acts = eng.prepare_inputs(xs)
    assert all(a.t.dtype == H for a in acts) and eng.pack_fwd.dtype == H
    scale, backoffs = 2.0 ** 16, 0
    while True:
        eng.flat.grad.zero_()
        loss, _ = eng.forward_backward(acts, labels, loss_scale=scale)
        if bool(torch.isfinite(eng.flat.grad).all()):
            break
        scale, backoffs = scale / 2, backoffs + 1
        assert backoffs <= 8, "fp16 gradients overflow even at 2^8"
    eng.flat.grad.div_(scale)
    torch.cuda.synchronize()
    print(f"fused loss scale 2^{int(math.log2(scale))} after {backoffs} back-offs")
    fe, ae = _grad_errs(model, oracle, ac)
    print(f"loss fused {float(loss):.4f} fp32 {float(loss_ref):.4f} fp16-autocast {float(loss_ac):.4f}; grad rel-L2 "
          f"median fused {fe[len(fe) // 2]:.4f} autocast {ae[len(ae) // 2]:.4f}")
    tol = max(0.05, 2 * abs(float(loss_ac) - float(loss_ref)))
    assert abs(float(loss) - float(loss_ref)) < tol * max(1.0, abs(float(loss_ref)))
    assert all(torch.isfinite(p.grad).all() for p in model.parameters())
    assert fe[len(fe) // 2] <= 2 * ae[len(ae) // 2] + 0.01
    assert fe[int(0.9 * len(fe))] <= 2 * ae[int(0.9 * len(ae))] + 0.02


def test_fp16_fixed_batch_training_with_loss_scale_backoff():
    """50 fp16 steps on one fixed batch with GradScaler dynamics: an oversized initial scale (2^30) overflows the fp16
    gradients, the step is skipped and the scale backs off until it fits; afterwards the loss stays finite and falls
    (memorisation)."""
    model = _sf()
    eng = FusedNet(model, DEV, compute_dtype=H)
    opt = FusedSGD(eng.flat, lr=0.02, momentum=0.9, weight_decay=1e-4, after_step=eng.pack)
    scaler = FusedGradScaler(init_scale=2.0 ** 30)
    xs = eng.prepare_inputs(_inputs(4, 8, 64, seed=9))
    labels = torch.tensor([1, 7, 3, 5], device=DEV)
    losses, skipped, scales = [], 0, []
    for _ in range(50):
        opt.zero_grad()
        loss, _ = eng.forward_backward(xs, labels, loss_scale=scaler.get_scale())
        scaler.step(opt)
        scaler.update()
        skipped += int(opt.step_was_skipped)
        scales.append(scaler.get_scale())
        losses.append(float(loss))
    print("skipped", skipped, "scales", scales[:12], "losses", " ".join("%.3f" % v for v in losses))
    assert skipped >= 1 and scales[-1] < 2.0 ** 30          # back-off exercised
    assert all(torch.isfinite(torch.tensor(losses)))
    assert min(losses[-10:]) < 0.5 * losses[0], losses
