"""Fused HIP executor vs the pure-PyTorch oracle (same weights, same bf16-rounded clip).

Checks one training micro-step of SlowFast-R50 and Slow-R50 at reduced resolution: loss, logits, every
parameter gradient (relative L2), BN running statistics, and that a few fused-SGD steps decrease the
loss on a fixed batch.
"""
import copy
import os

import pytest
import torch
import torch.nn.functional as F

from pytorchvideo_accelerate_amd.models import reference as R
from pytorchvideo_accelerate_amd.models.fused import FusedNet
from pytorchvideo_accelerate_amd.ops.optim import FusedSGD

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _inputs(slowfast, N=2, T=8, S=64, alpha=4, seed=0):
    g = torch.Generator().manual_seed(seed)
    fast = torch.randn(N, 3, T, S, S, generator=g).to(torch.bfloat16).float()
    if not slowfast:
        return [fast]
    idx = torch.linspace(0, T - 1, T // alpha).long()
    return [fast[:, :, idx].contiguous(), fast]


def _build(slowfast, classes=10):
    torch.manual_seed(0)
    if slowfast:
        return R.create_slowfast(50, classes, head_pool_kernel_sizes=((2, 2, 2), (8, 2, 2)), dropout_rate=0.0)
    return R.create_resnet(50, classes, head_pool_kernel_size=(1, 2, 2), dropout_rate=0.0)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("slowfast", [True, False])
def test_fused_step_matches_oracle(slowfast):
    model = _build(slowfast)
    oracle_init = copy.deepcopy(model)
    oracle = copy.deepcopy(model).to(DEV).train()
    xs = _inputs(slowfast)
    labels = torch.tensor([1, 7], device=DEV)
    # oracle fp32
    out_ref = oracle([x.to(DEV) for x in xs] if slowfast else xs[0].to(DEV))
    loss_ref = F.cross_entropy(out_ref, labels)
    loss_ref.backward()
    # fused
    eng = FusedNet(model, DEV)
    acts = eng.prepare_inputs(xs)
    loss, logits = eng.forward_backward(acts, labels)
    torch.cuda.synchronize()
    # Stock PyTorch bf16 autocast on the same weights/inputs = the bf16 noise floor of a 50-layer net
    # with batch statistics over tiny tensors (errors compound through every BN).
    ac = copy.deepcopy(oracle_init).to(DEV).train()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out_ac = ac([x.to(DEV) for x in xs] if slowfast else xs[0].to(DEV))
    loss_ac = F.cross_entropy(out_ac.float(), labels)
    loss_ac.backward()
    # One autocast run is a single sample of that noise: equally valid bf16 executions that differ only in
    # launch configuration (i.e. fp32 summation order of the BN partial sums) land up to ~4 % apart at this
    # size (scripts/debug_direct.py @ a59cdac: 2.246 / 2.258 / 2.320 / 2.338 for four configuration mixes; random-init
    # BN nets amplify bf16 rounding with depth), so the loss floor is 8 %.
    tol = max(8e-2, 2 * abs(loss_ac.item() - loss_ref.item()))
    assert abs(loss.item() - loss_ref.item()) < tol * max(1.0, abs(loss_ref.item()))
    ref_params = dict(oracle.named_parameters())
    ac_params = dict(ac.named_parameters())
    fe = sorted(_rel(p.grad, ref_params[n].grad) for n, p in model.named_parameters())
    ae = sorted(_rel(ac_params[n].grad, ref_params[n].grad) for n, _ in model.named_parameters())
    assert fe[len(fe) // 2] <= 1.5 * ae[len(ae) // 2] + 0.02, (fe[len(fe) // 2], ae[len(ae) // 2])
    ref_bufs = dict(oracle.named_buffers())
    ac_bufs = dict(ac.named_buffers())
    for n, b in model.named_buffers():
        if n.endswith("running_var"):
            assert _rel(b, ref_bufs[n]) <= 2 * _rel(ac_bufs[n], ref_bufs[n]) + 0.02, n
        if n.endswith("num_batches_tracked"):
            assert int(b) == int(ref_bufs[n]), n


@pytest.mark.parametrize("slowfast", [True, False])
def test_fused_eval_matches_oracle(slowfast):
    model = _build(slowfast)
    # make running stats non-trivial
    for m in model.modules():
        if isinstance(m, torch.nn.BatchNorm3d):
            m.running_mean.uniform_(-0.1, 0.1)
            m.running_var.uniform_(0.5, 1.5)
    oracle = copy.deepcopy(model).to(DEV).eval()
    xs = _inputs(slowfast, seed=1)
    with torch.no_grad():
        ref = oracle([x.to(DEV) for x in xs] if slowfast else xs[0].to(DEV))
    eng = FusedNet(model, DEV)
    out = eng.forward_eval(eng.prepare_inputs(xs))
    assert _rel(out, ref) < 5e-2


def test_fused_sgd_tracks_torch_training():
    model = _build(True)
    oracle = copy.deepcopy(model).to(DEV).train()
    eng = FusedNet(model, DEV)
    opt = FusedSGD(eng.flat, lr=0.01, momentum=0.9, weight_decay=1e-4, after_step=eng.pack)
    ropt = torch.optim.SGD(oracle.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    xs = _inputs(True, N=4, seed=3)
    acts = eng.prepare_inputs(xs)
    labels = torch.tensor([3, 4, 5, 6], device=DEV)
    losses, ref_losses = [], []
    for _ in range(6):
        opt.zero_grad()
        loss, _ = eng.forward_backward(acts, labels)
        opt.step()
        losses.append(loss.item())
        ropt.zero_grad()
        rl = F.cross_entropy(oracle([x.to(DEV) for x in xs]), labels)
        rl.backward()
        ropt.step()
        ref_losses.append(rl.item())
    # fused bf16 SGD tracks fp32 torch SGD over the first steps and decreases the loss
    assert losses[1] < losses[0], (losses, ref_losses)
    for a, b in zip(losses[:3], ref_losses[:3]):
        assert abs(a - b) < 0.2 * abs(b) + 0.05, (losses, ref_losses)


def test_fused_sgd_matches_torch_sgd():
    model = _build(False)
    ref = copy.deepcopy(model).to(DEV)
    eng = FusedNet(model, DEV)
    opt = FusedSGD(eng.flat, lr=0.1, momentum=0.9, weight_decay=1e-4)
    ropt = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    g = torch.Generator(device="cpu").manual_seed(0)
    for _ in range(3):
        for (n, p), (_, q) in zip(model.named_parameters(), ref.named_parameters()):
            gr = torch.randn(p.shape, generator=g).to(DEV)
            eng.flat.gview(p).copy_(gr)
            q.grad = gr.clone()
        opt.step()
        ropt.step()
    for (n, p), (_, q) in zip(model.named_parameters(), ref.named_parameters()):
        torch.testing.assert_close(p.data, q.data, rtol=1e-5, atol=1e-6)
    sd = opt.state_dict()
    assert "momentum_buffer" in sd["state"][0]


def test_deterministic_mode_is_bitwise_reproducible():
    """deterministic=True: slab wgrad reduction + fixed-order BN reductions -> identical gradients run to run.
    Against the default mode (s2d stems, wgrad atomics) only the loss is compared: on this tiny config bf16
    rounding differences are amplified through 50 batch-statistics BNs (see the oracle tests above)."""
    xs = _inputs(True, N=2, T=8, S=64)
    labels = torch.tensor([3, 5], device=DEV)
    grads, losses = [], []
    for det in (True, True, False):
        eng = FusedNet(_build(True), DEV, deterministic=det)
        assert eng.input_s2d is not det
        loss, _ = eng.forward_backward(eng.prepare_inputs(xs), labels)
        torch.cuda.synchronize()
        grads.append(eng.flat.grad.clone())
        losses.append(loss.item())
    assert torch.equal(grads[0], grads[1]) and losses[0] == losses[1]
    assert abs(losses[2] - losses[0]) < 0.05 * abs(losses[0])


def test_two_stream_step_matches_single_stream():
    """The fast pathway on its own HIP stream (after the autotuning step) gives the same loss and gradients
    as the single-stream schedule on the same inputs (up to fp32-atomic ordering in the weight gradients)."""
    model = _build(True)
    eng = FusedNet(model, DEV)
    acts = eng.prepare_inputs(_inputs(True, seed=3))
    labels = torch.tensor([2, 5], device=DEV)
    eng.forward_backward(acts, labels)          # tuning step, single stream
    assert eng._ms_ok and eng._ms_warm and eng._ms_active()
    res = {}
    for ms in (False, True):
        eng._ms_ok = ms
        loss, logits = eng.forward_backward(acts, labels, accumulate=False)
        torch.cuda.synchronize()
        res[ms] = (float(loss), logits.clone(), eng.flat.grad.clone())
    (l0, g0_logits, g0), (l1, g1_logits, g1) = res[False], res[True]
    assert abs(l0 - l1) < 1e-4 * max(1.0, abs(l0))
    assert _rel(g1_logits, g0_logits) < 1e-4
    assert _rel(g1, g0) < 1e-3


def test_persistent_tune_cache_reused_and_invalidated(tmp_path, monkeypatch):
    """A second executor on the same build/device/dtype restores every autotuner choice from the table the first
    one wrote and times nothing; a different build stamp (rebuilt .so) gets a fresh table and tunes again."""
    from pytorchvideo_accelerate_amd.ops import tune
    monkeypatch.setenv("PVA_TUNE_CACHE", str(tmp_path))
    xs = _inputs(True)
    labels = torch.tensor([1, 7], device=DEV)
    e1 = FusedNet(_build(True), DEV)
    l1, _ = e1.forward_backward(e1.prepare_inputs(xs), labels)
    e1.forward_eval(e1.prepare_inputs(xs))
    assert e1.tuner.tuned > 0 and os.path.exists(e1.tune_store.path)
    e2 = FusedNet(_build(True), DEV)
    assert len(e2.tuner.cache) == len(e1.tuner.cache) and len(e2.wtune) == len(e1.wtune)
    l2, _ = e2.forward_backward(e2.prepare_inputs(xs), labels)
    e2.forward_eval(e2.prepare_inputs(xs))
    assert e2.tuner.tuned == 0
    assert torch.isfinite(l2) and abs(l1.item() - l2.item()) < 0.05 * abs(l1.item())
    real = tune.TuneStore.build_ident
    monkeypatch.setattr(tune.TuneStore, "build_ident", staticmethod(lambda d, t: dict(real(d, t), so="stale")))
    e3 = FusedNet(_build(True), DEV)
    assert len(e3.tuner.cache) == 0
    e3.forward_backward(e3.prepare_inputs(xs), labels)
    assert e3.tuner.tuned > 0


def test_narrow_fused_backward_matches_unfused(monkeypatch):
    """The fused narrow conv_c backward (fast res2: BN apply + weight gradient + input gradient in one pass,
    csrc/kernels/narrow_bwd.hip), with and without the narrow BN fold of the forward (arm narrow_fold), against the
    three-kernel unfolded path it replaces (narrow_bwd=0), deterministic mode: loss, every gradient and the BN
    running statistics within bf16 re-association noise."""
    model = _build(True)
    xs = _inputs(True, N=2, T=16, S=96, seed=3)
    labels = torch.tensor([2, 5], device=DEV)
    runs = []
    for flag, fold in (("1", "1"), ("1", "0"), ("0", "0")):
        monkeypatch.setenv("PVA_ARMS", f"narrow_bwd={flag},narrow_fold={fold}")
        m = copy.deepcopy(model)
        eng = FusedNet(m, DEV, deterministic=True)
        blocks = [b for paths, _ in eng.stages for p in paths for b in getattr(p, "blocks", [])]
        assert any(b.narrow_c for b in blocks) == (flag == "1")
        assert any(b.narrow_fold for b in blocks) == (fold == "1")
        loss, _ = eng.forward_backward(eng.prepare_inputs(xs), labels)
        torch.cuda.synchronize()
        runs.append((float(loss), {n: p.grad.detach().clone() for n, p in m.named_parameters()},
                     {n: b.detach().clone() for n, b in m.named_buffers()}))
    l0, g0, b0 = runs[-1]
    # fused unfolded: the same forward, the backward re-associated -> loss identical, gradients within 2e-2
    l1, g1, b1 = runs[1]
    assert abs(l1 - l0) < 1e-6 * max(1.0, abs(l0)), (l1, l0)
    worst = max((_rel(g1[n], g0[n]), n) for n in g0 if g0[n].norm() > 0)
    assert worst[0] < 2e-2, worst
    # folded: the unit output comes from a recomputing kernel and the BN statistics from a statistics-only pass —
    # other bf16 roundings of the same forward.  At this random-init whole-net shape the backward is chaotic (every
    # fused variant, unfolded included, sits at median rel-L2 ~1.2 from the fp32 oracle: scripts/diag_narrow.py @ a59cdac), so
    # only the loss and the running statistics are compared here; the folded backward is gated block-level
    # (tests/test_blocks_gpu.py::test_fast_res2_narrow) against the fp32 oracle.
    lf, gf, bf = runs[0]
    assert abs(lf - l0) < 1e-2 * max(1.0, abs(l0)), (lf, l0)
    # a running mean is measured on the scale of its feature's spread (relative to ~0 means it is noise-dominated)
    def err(b, ref, n):
        if n.endswith("running_mean"):
            return float((b[n] - ref[n]).norm() / ref[n[:-4] + "var"].clamp_min(0).sqrt().norm())
        return _rel(b[n], ref[n])
    names = [n for n in b0 if b0[n].dtype.is_floating_point]
    for n in names:
        assert err(b1, b0, n) < 1e-2, (n, err(b1, b0, n))
    # the folded forward's statistics: against the fp32 oracle, within twice the unfolded bf16 path's own distance
    oracle = copy.deepcopy(model).to(DEV).train()
    with torch.no_grad():
        oracle([x.to(DEV) for x in xs])
    bo = {n: b.detach() for n, b in oracle.named_buffers()}
    for n in names:
        ef, e0 = err(bf, bo, n), err(b0, bo, n)
        assert ef < 2 * e0 + 5e-3, (n, ef, e0)
