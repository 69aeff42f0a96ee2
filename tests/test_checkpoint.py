"""Checkpoint layout parity: directories written by this engine load with the installed
``accelerate.Accelerator.load_state`` and vice versa."""
import copy
import os

import pytest
import torch

from pytorchvideo_accelerate_amd.ckpt.state import latest_checkpoint, load_state, save_state
from pytorchvideo_accelerate_amd.engine.accelerator import GlobalRateScheduler
from pytorchvideo_accelerate_amd.models import reference as R
from pytorchvideo_accelerate_amd.models.fused import FlatParams
from pytorchvideo_accelerate_amd.ops.optim import FusedSGD

accelerate = pytest.importorskip("accelerate")


def _small_model(seed=0):
    torch.manual_seed(seed)
    return R.create_resnet(50, 5, head_pool_kernel_size=(1, 2, 2))


def _ours(seed=0, steps=2):
    m = _small_model(seed)
    flat = FlatParams(list(reversed(list(m.named_parameters()))), torch.device("cpu"))
    opt = FusedSGD(flat, lr=0.1, momentum=0.9, weight_decay=1e-4, params=list(m.parameters()))
    sch = GlobalRateScheduler(torch.optim.lr_scheduler.CosineAnnealingLR(opt, 10), opt, 1)
    g = torch.Generator().manual_seed(1)
    for _ in range(steps):
        flat.grad.copy_(torch.randn(flat.grad.shape, generator=g))
        opt.step()
        sch.step()
    # non-trivial BN buffers
    for b in m.buffers():
        if b.dtype == torch.float32:
            b.uniform_(0.5, 1.5)
    return m, opt, sch


def test_ours_loads_in_accelerate(tmp_path):
    m, opt, sch = _ours()
    d = str(tmp_path / "epoch_0")
    save_state(d, m, [opt], [sch], [sch], step=7)
    assert sorted(os.listdir(d)) == sorted(["model.safetensors", "optimizer.bin", "scheduler.bin",
                                            "custom_checkpoint_0.pkl", "random_states_0.pkl", ".pva_complete"])
    acc = accelerate.Accelerator(cpu=True)
    m2 = _small_model(seed=3)
    o2 = torch.optim.SGD(m2.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    s2 = torch.optim.lr_scheduler.CosineAnnealingLR(o2, 10)
    m2, o2, s2 = acc.prepare(m2, o2, s2)
    acc.register_for_checkpointing(s2)
    acc.load_state(d)
    for (n, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        torch.testing.assert_close(a, b, msg=n)
    for p, q in zip(m.parameters(), m2.parameters()):
        torch.testing.assert_close(opt.state[p]["momentum_buffer"], o2.state[q]["momentum_buffer"].cpu())
    assert s2.scheduler.last_epoch == sch.scheduler.last_epoch == 2
    assert acc.step == 7


def test_accelerate_checkpoint_loads_in_ours(tmp_path):
    acc = accelerate.Accelerator(cpu=True)
    m = _small_model(seed=4)
    o = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    s = torch.optim.lr_scheduler.CosineAnnealingLR(o, 10)
    m, o, s = acc.prepare(m, o, s)
    acc.register_for_checkpointing(s)
    for p in m.parameters():
        p.grad = torch.randn_like(p)
    o.step()
    s.step()
    d = str(tmp_path / "step_3")
    acc.save_state(d)
    m2, o2, s2 = _ours(seed=9, steps=0)
    ov = load_state(d, m2, [o2], [s2], [s2])
    for (n, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        torch.testing.assert_close(a, b, msg=n)
    for p, q in zip(m.parameters(), m2.parameters()):
        torch.testing.assert_close(o.state[p]["momentum_buffer"], o2.state[q]["momentum_buffer"])
    assert s2.scheduler.last_epoch == s.scheduler.last_epoch
    assert "step" in ov
    # the loaded momentum lives in the flat buffer: one more fused step equals one more torch step
    g = [torch.randn_like(p) for p in m.parameters()]
    for p, q, gg in zip(m.parameters(), m2.parameters(), g):
        p.grad = gg.clone()
        o2.flat.gview(q).copy_(gg)
    o.step()
    o2.step()
    for p, q in zip(m.parameters(), m2.parameters()):
        torch.testing.assert_close(p.data, q.data, rtol=1e-5, atol=1e-6)


def test_module_prefix_stripped_and_latest(tmp_path):
    from safetensors.torch import save_file
    m = _small_model()
    d = tmp_path / "step_5"
    d.mkdir()
    save_file({"module." + k: v.contiguous() for k, v in m.state_dict().items()}, str(d / "model.safetensors"))
    m2 = _small_model(seed=1)
    from pytorchvideo_accelerate_amd.ckpt.state import load_model_state
    load_model_state(m2, str(d))
    for a, b in zip(m.state_dict().values(), m2.state_dict().values()):
        torch.testing.assert_close(a, b)
    e = tmp_path / "epoch_1"
    e.mkdir()
    save_file({k: v.contiguous() for k, v in m.state_dict().items()}, str(e / "model.safetensors"))
    # foreign / unfinished directories (no completion marker) are never auto-resumed from
    assert latest_checkpoint(str(tmp_path)) is None
    (d / ".pva_complete").write_text("{}")
    (e / ".pva_complete").write_text("{}")
    os.utime(str(d), (1, 1))
    assert latest_checkpoint(str(tmp_path)) == str(e)
    assert latest_checkpoint(str(tmp_path / "nope")) is None


def test_crash_mid_save_resumes_from_previous_complete(tmp_path, monkeypatch):
    """A save that dies half-way leaves no directory that auto-resume would pick (atomic rename + marker)."""
    from pytorchvideo_accelerate_amd.ckpt.state import InjectedSaveFault, is_complete
    m, opt, sch = _ours()
    save_state(str(tmp_path / "step_2"), m, [opt], [sch], [sch], step=2)
    monkeypatch.setenv("PVA_FAULT", "save=4")
    with pytest.raises(InjectedSaveFault):
        save_state(str(tmp_path / "step_4"), m, [opt], [sch], [sch], step=4)
    assert not (tmp_path / "step_4").exists() and (tmp_path / "step_4.tmp" / "model.safetensors").exists()
    assert latest_checkpoint(str(tmp_path)) == str(tmp_path / "step_2") and is_complete(str(tmp_path / "step_2"))
    # the restarted run passes the hook (marker file) and the retried save completes, replacing the leftover
    save_state(str(tmp_path / "step_4"), m, [opt], [sch], [sch], step=4)
    assert is_complete(str(tmp_path / "step_4")) and not (tmp_path / "step_4.tmp").exists()
    assert latest_checkpoint(str(tmp_path)) == str(tmp_path / "step_4")
    # re-saving into an existing complete directory (the final save) swaps it atomically
    m2, _, _ = _ours(seed=5)
    save_state(str(tmp_path / "step_4"), m2, [opt], [sch], [sch], step=4)
    from pytorchvideo_accelerate_amd.ckpt.state import load_model_state
    m3 = _small_model(seed=7)
    load_model_state(m3, str(tmp_path / "step_4"))
    for a, b in zip(m2.state_dict().values(), m3.state_dict().values()):
        torch.testing.assert_close(a, b)
    assert not (tmp_path / "step_4.old").exists()
