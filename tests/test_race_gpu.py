"""Race detection for the production multi-stream schedule (verdict r5 item 4, SURVEY.md §5 "Race detection").

* The dependency checker (``utils/depcheck.py``) follows every kernel launch, event record and stream wait of the
  shipped configuration (two pathway streams + per-lane weight-gradient streams, autotuned kernels, s2d stems) and
  reports any cross-stream read/write without an ordering event: the default schedule must be hazard-free, and
  dropping round 5's missing join (the fast stage of the fusion-less res5 stage reading the head's pooled-gradient
  scatter from the main stream, commit ebb2a15) must be reported deterministically.
* The reproducible schedule (``FusedNet(reproducible=True)``): the same streams, s2d stems and a *fixed* table of
  kernel choices, with fixed-order (slab) reductions in place of the weight-gradient atomics — two runs of the
  multi-stream step give bitwise-identical gradients at B=16.
"""
import pytest
import torch

from pytorchvideo_accelerate_amd.models import reference as R
from pytorchvideo_accelerate_amd.models.fused import FusedNet
from pytorchvideo_accelerate_amd.utils import depcheck

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _net(B=2, T=8, S=64, **kw):
    torch.manual_seed(0)
    model = R.create_slowfast(50, 10, head_pool_kernel_sizes=((T // 4, S // 32, S // 32), (T, S // 32, S // 32)),
                              dropout_rate=0.0)
    eng = FusedNet(model, DEV, **kw)
    g = torch.Generator().manual_seed(1)
    fast = torch.randn(B, 3, T, S, S, generator=g)
    xs = [fast[:, :, torch.linspace(0, T - 1, T // 4).long()].contiguous(), fast]
    labels = torch.randint(0, 10, (B,), generator=g).to(DEV)
    return eng, eng.prepare_inputs(xs), labels


def _checked_step(eng, acts, labels):
    chk = depcheck.install(eng)
    try:
        with chk.watching():
            eng.forward_backward(acts, labels, accumulate=False)
            torch.cuda.synchronize()
    finally:
        depcheck.uninstall(chk)
    return chk


def test_production_schedule_has_no_cross_stream_hazard():
    eng, acts, labels = _net()
    eng.forward_backward(acts, labels, accumulate=False)   # autotuning step (one stream)
    torch.cuda.synchronize()
    assert eng._ms_ok, "the multi-stream schedule must be on for this test"
    chk = _checked_step(eng, acts, labels)
    assert eng._ms_active() and len(chk.count) >= 3, f"streams seen: {len(chk.count)}"
    assert chk.launches > 300
    assert not chk.hazards, "\n".join(map(str, chk.hazards[:10]))


def test_dropped_head_scatter_join_is_reported():
    eng, acts, labels = _net()
    eng.forward_backward(acts, labels, accumulate=False)
    torch.cuda.synchronize()
    eng.debug_skip_joins = {"head_scatter"}
    chk = _checked_step(eng, acts, labels)
    eng.debug_skip_joins = set()
    assert chk.hazards, "the dropped join must be reported"
    assert any(h.kind == "RAW" and h.other_fn == "avgpool_bwd" for h in chk.hazards), \
        "\n".join(map(str, chk.hazards[:10]))


def test_checker_sees_missing_wait_in_a_two_stream_toy():
    """Unit check of the clock model: a read on stream B of a buffer written on stream A needs A's event."""
    chk = depcheck.DepChecker()
    a = torch.cuda.Stream()
    b = torch.cuda.Stream()
    x = torch.zeros(1024, device=DEV)
    y = torch.zeros(1024, device=DEV)
    fake = lambda *args, **kw: None   # noqa: E731
    with chk.watching():
        with torch.cuda.stream(a):
            chk.on_launch("bn_act", fake, (x, 4, y, 4, x, x, 0, 1, 4), {})   # writes y on a
        with torch.cuda.stream(b):
            chk.on_launch("bn_act", fake, (y, 4, x, 4, y, y, 0, 1, 4), {})   # reads y on b: RAW, no wait
        assert {h.kind for h in chk.hazards} == {"RAW", "WAR"}
        chk.hazards.clear()
        ev = torch.cuda.Event()
        ev.record(a)
        b.wait_event(ev)
        with torch.cuda.stream(b):
            chk.on_launch("bn_act", fake, (y, 4, x, 4, y, y, 0, 1, 4), {})
        assert not chk.hazards


def test_reproducible_production_schedule_is_bitwise_stable():
    """B=16, both pathway streams and the weight-gradient streams active: two steps at the same weights and inputs
    give bitwise-identical loss, logits and flat gradient."""
    eng, acts, labels = _net(B=16, reproducible=True)
    eng.forward_backward(acts, labels, accumulate=False)   # tuning step: fixes the kernel choices
    torch.cuda.synchronize()
    runs = []
    for _ in range(2):
        loss, logits = eng.forward_backward(acts, labels, accumulate=False)
        torch.cuda.synchronize()
        runs.append((loss.clone(), logits.clone(), eng.flat.grad.clone()))
    assert eng._ms_active() and eng._side is not None and all(st is not None for st in eng._wst), \
        "the multi-stream schedule (side lane + both weight-gradient streams) must have run"
    (l0, z0, g0), (l1, z1, g1) = runs
    assert torch.isfinite(g0).all()
    assert torch.equal(l0, l1) and torch.equal(z0, z1)
    assert torch.equal(g0, g1), f"{(g0 != g1).sum().item()} gradient entries differ"
