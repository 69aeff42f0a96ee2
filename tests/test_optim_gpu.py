"""Fused SGD kernel paths used by fp16 loss scaling: device-side non-finite check + skipped update."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def test_nonfinite_check_and_skipped_sgd():
    from pytorchvideo_accelerate_amd.ops._ext import require
    C = require()
    n = 1000003                      # odd length: exercises the scalar tail
    g = torch.randn(n, device=DEV)
    p = torch.randn(n, device=DEV)
    buf = torch.zeros(n, device=DEV)
    lr = torch.full((1,), 0.1, device=DEV)
    flag = torch.zeros(1, dtype=torch.int32, device=DEV)
    C.nonfinite_check(g, 1.0 / 1024, flag)
    assert int(flag) == 0
    p0 = p.clone()
    C.sgd_momentum(p, g, buf, lr, 0.9, 1e-4, 1.0 / 1024, 1, None, flag)
    torch.testing.assert_close(p, p0 - 0.1 * (g / 1024 + 1e-4 * p0), rtol=1e-5, atol=1e-6)
    for bad_at in (5, n - 1):        # vector body and tail
        g2 = g.clone()
        g2[bad_at] = float("inf") if bad_at == 5 else float("nan")
        flag.zero_()
        C.nonfinite_check(g2, 1.0, flag)
        assert int(flag) == 1
        p1, b1 = p.clone(), buf.clone()
        C.sgd_momentum(p, g2, buf, lr, 0.9, 1e-4, 1.0, 0, None, flag)
        assert torch.equal(p, p1) and torch.equal(buf, b1)
    # overflow produced by the scale itself (finite grads * huge scale)
    flag.zero_()
    C.nonfinite_check(torch.full((64,), 3e38, device=DEV), 10.0, flag)
    assert int(flag) == 1
