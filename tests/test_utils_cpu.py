"""CPU tests of the observability / debug utilities."""
import time

import pytest
import torch

from pytorchvideo_accelerate_amd.models.fused import FlatParams
from pytorchvideo_accelerate_amd.utils.debug import GradChecker, debug_env
from pytorchvideo_accelerate_amd.utils.metrics import Accuracy
from pytorchvideo_accelerate_amd.utils.profiling import StepTimer


def test_step_timer_phases_and_quantiles():
    t = StepTimer(torch.device("cpu"))
    for i in range(10):
        t.begin_step()
        with t.host("data"):
            time.sleep(0.001)
        with t.phase("fwd_bwd"):
            time.sleep(0.002 + 0.001 * (i == 9))
        t.end_step(clips=4)
    s = t.summary()
    assert s["data_wait_ms"] >= 1.0 and s["fwd_bwd_ms"] >= 2.0 and s["comm_ms"] == 0.0
    assert s["step_time_p90_ms"] >= s["step_time_ms"] > 3.0 and 0 < s["clips_per_sec"] < 4 / 0.003


def test_grad_checker_names_bad_params():
    net = torch.nn.Sequential(torch.nn.Linear(3, 4), torch.nn.Linear(4, 2))
    flat = FlatParams(list(net.named_parameters()), torch.device("cpu"))
    chk = GradChecker(flat)
    flat.grad.normal_()
    chk.check(0)
    flat.gview(net[1].weight)[0, 1] = float("nan")
    assert chk.bad_params() == ["1.weight"]
    with pytest.raises(FloatingPointError, match="1.weight"):
        chk.check(5)
    assert debug_env()["AMD_SERIALIZE_KERNEL"] == "3"


def test_accuracy_metric():
    m = Accuracy()
    logits = torch.tensor([[0.1, 0.9], [0.8, 0.2], [0.3, 0.7]])
    assert m(logits, torch.tensor([1, 1, 1])).item() == pytest.approx(2 / 3)
    m.update(torch.tensor([0, 0]), torch.tensor([0, 1]))
    assert m.compute().item() == pytest.approx(3 / 5)
    m.reset()
    assert m.compute().item() == 0.0


def test_arms_single_knob(monkeypatch):
    """Decided A/B arms live behind one knob (PVA_ARMS); defaults are the shipped arms; typos raise."""
    from pytorchvideo_accelerate_amd.utils import arms
    monkeypatch.delenv("PVA_ARMS", raising=False)
    assert arms.arm("stem_pair") == 1 and arms.arm("bn_fold_min_c") == 16 and arms.selected() == {}
    monkeypatch.setenv("PVA_ARMS", "stem_pair=0, bn_fold_min_c=8")
    assert arms.arm("stem_pair") == 0 and arms.arm("bn_fold_min_c") == 8
    assert arms.selected() == {"stem_pair": 0, "bn_fold_min_c": 8}
    assert arms.arms_spec(side_fuse=False) == "stem_pair=0,bn_fold_min_c=8,side_fuse=0"
    monkeypatch.setenv("PVA_ARMS", "stem_pari=0")
    with pytest.raises(ValueError):
        arms.arm("stem_pair")


def test_fault_spec(monkeypatch):
    from pytorchvideo_accelerate_amd.utils.misc import fault_at
    monkeypatch.setenv("PVA_FAULT", "step=3,save=4")
    assert fault_at("step") == 3 and fault_at("save") == 4
    monkeypatch.delenv("PVA_FAULT")
    assert fault_at("step") is None
