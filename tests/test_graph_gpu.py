"""HIP-graph replay of the fused training step (engine/graph.py): a captured forward+backward+SGD step gives the
same loss and parameter update as the eager step from the same state, and replays draw fresh dropout keys."""
import pytest
import torch

from pytorchvideo_accelerate_amd.models import reference as R
from pytorchvideo_accelerate_amd.models.fused import FusedNet
from pytorchvideo_accelerate_amd.ops.optim import FusedSGD

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


def test_graph_step_matches_eager():
    from pytorchvideo_accelerate_amd.engine.graph import GraphedStep
    torch.manual_seed(0)
    model = R.create_slowfast(50, 10, head_pool_kernel_sizes=((2, 2, 2), (8, 2, 2)), dropout_rate=0.5)
    eng = FusedNet(model, DEV)
    opt = FusedSGD(eng.flat, lr=0.05, momentum=0.9, weight_decay=1e-4, after_step=eng.pack)
    g = torch.Generator().manual_seed(3)
    fast = torch.randn(2, 3, 8, 64, 64, generator=g).to(torch.bfloat16).float()
    xs = eng.prepare_inputs([fast[:, :, torch.linspace(0, 7, 2).long()].contiguous(), fast])
    labels = torch.tensor([2, 5], device=DEV)
    for _ in range(2):                       # autotuning step, then the optimizer's state-binding step
        opt.zero_grad()
        eng.forward_backward(xs, labels)
        opt.step()
    torch.cuda.synchronize()
    bufs = list(model.buffers())
    snap = (eng.flat.data.clone(), opt.buf.clone(), eng._seed_dev.clone(), [b.clone() for b in bufs])

    def restore():
        eng.flat.data.copy_(snap[0]); opt.buf.copy_(snap[1]); eng._seed_dev.copy_(snap[2])
        for b, s in zip(bufs, snap[3]):
            b.copy_(s)
        eng.pack()

    opt.zero_grad()
    loss_e, _ = eng.forward_backward(xs, labels)
    opt.step()
    torch.cuda.synchronize()
    le, pe = float(loss_e), eng.flat.data.clone()
    restore()
    gs = GraphedStep(eng, opt)
    loss_g, _ = gs(xs, labels, accumulate=False, optimizer_step=True)   # capture + first replay
    torch.cuda.synchronize()
    lg, pg = float(loss_g), eng.flat.data.clone()
    assert len(gs.graphs) == 1
    assert abs(le - lg) < 2e-3 * max(1.0, abs(le)), (le, lg)
    step_e, step_g = pe - snap[0], pg - snap[0]
    assert _rel(step_g, step_e) < 2e-2                      # the same SGD update (fp32-atomic wgrad order aside)
    seed1 = int(eng._seed_dev.item())
    gs(xs, labels, accumulate=False, optimizer_step=True)  # replay: the dropout key advances on the device
    torch.cuda.synchronize()
    assert int(eng._seed_dev.item()) != seed1 and len(gs.graphs) == 1
