"""fp16 dynamic loss scaling of the fused path (FusedGradScaler; reference recipe run_slowfast_r50.sh:7,
accelerate/torch GradScaler semantics): skipped steps on overflow (parameters, momentum and the LR
schedule untouched), backoff / growth, and scaler.pt checkpoint round trip."""
import torch

from pytorchvideo_accelerate_amd.ckpt.state import load_state, save_state
from pytorchvideo_accelerate_amd.engine.accelerator import GlobalRateScheduler
from pytorchvideo_accelerate_amd.models.fused import FlatParams
from pytorchvideo_accelerate_amd.ops.optim import FusedGradScaler, FusedSGD


def _setup():
    torch.manual_seed(0)
    net = torch.nn.Linear(4, 3)
    flat = FlatParams(list(reversed(list(net.named_parameters()))), torch.device("cpu"))
    opt = FusedSGD(flat, lr=0.1, momentum=0.9, weight_decay=1e-4, params=list(net.parameters()))
    sched = GlobalRateScheduler(torch.optim.lr_scheduler.CosineAnnealingLR(opt, 10), opt, 1)
    return net, flat, opt, sched


def _step(flat, opt, sched, scaler, grad):
    flat.grad.copy_(grad * scaler.get_scale())     # backward of loss * scale
    scaler.step(opt)
    scaler.update()
    sched.step()


def test_overflow_skips_step_and_scheduler_then_recovers():
    net, flat, opt, sched = _setup()
    scaler = FusedGradScaler(init_scale=2.0 ** 16, growth_interval=3)
    g = torch.randn(flat.numel)
    p0 = flat.data.clone()
    bad = g.clone()
    bad[1] = float("inf")
    _step(flat, opt, sched, scaler, bad)
    assert opt.step_was_skipped and torch.equal(flat.data, p0)
    assert scaler.get_scale() == 2.0 ** 15
    assert sched.scheduler.last_epoch == 0 and opt.param_groups[0]["lr"] == 0.1   # scheduler skipped too
    assert opt._first                                   # momentum not initialised by the skipped step
    # clean steps: the first one applies the unscaled gradient (p -= lr * (g + wd p))
    _step(flat, opt, sched, scaler, g)
    torch.testing.assert_close(flat.data, p0 - 0.1 * (g + 1e-4 * p0), rtol=1e-5, atol=1e-6)
    for _ in range(2):
        _step(flat, opt, sched, scaler, g)
        assert not opt.step_was_skipped
    assert scaler.get_scale() == 2.0 ** 16              # grew after growth_interval clean steps
    assert sched.scheduler.last_epoch == 3


def test_nan_is_overflow_and_state_dict_round_trip(tmp_path):
    net, flat, opt, sched = _setup()
    scaler = FusedGradScaler(init_scale=1024.0)
    g = torch.full((flat.numel,), float("nan"))
    _step(flat, opt, sched, scaler, g)
    assert opt.step_was_skipped and scaler.get_scale() == 512.0
    _step(flat, opt, sched, scaler, torch.ones(flat.numel))
    sd = scaler.state_dict()
    assert set(sd) == {"scale", "growth_factor", "backoff_factor", "growth_interval", "_growth_tracker"}
    assert sd["_growth_tracker"] == 1
    # torch's GradScaler accepts the same state (scaler.pt interop)
    ts = torch.amp.GradScaler("cpu")
    ts.load_state_dict(sd)
    assert ts.state_dict()["scale"] == 512.0
    save_state(str(tmp_path / "ck"), net, [opt], [sched], [], scaler=scaler)
    assert (tmp_path / "ck" / "scaler.pt").exists()
    s2 = FusedGradScaler()
    load_state(str(tmp_path / "ck"), net, [opt], [sched], [], scaler=s2)
    assert s2.state_dict() == sd
