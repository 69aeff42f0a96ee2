"""HIP classification head (csrc/kernels/head.hip) vs a float64 PyTorch reference of the same op:
dropout -> per-position Linear -> position mean -> softmax cross-entropy, forward + backward, and the eval
argmax/correct counts (reference run.py:109,254,297)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _C():
    from pytorchvideo_accelerate_amd.ops._ext import require
    return require()


def _ref(feat, W, b, labels, mask, p, scale):
    f = feat.double().requires_grad_(True)
    Wd = W.double().requires_grad_(True)
    bd = b.double().requires_grad_(True)
    x = f * mask.double() / (1 - p) if p > 0 else f
    logits = (x @ Wd.t() + bd).mean(1)            # per-position linear, then position mean
    loss = F.cross_entropy(logits, labels)
    (loss * scale).backward()
    return logits.detach(), loss.detach(), Wd.grad, bd.grad, f.grad


def _run(N, P, Cf, K, p, scale=0.5, seed=1234, beta=0.0):
    C = _C()
    g = torch.Generator(device="cpu").manual_seed(N * 131 + K)
    feat = torch.randn(N, P, Cf, generator=g).to(DEV)
    W = (torch.randn(K, Cf, generator=g) * 0.05).to(DEV)
    b = (torch.randn(K, generator=g) * 0.1).to(DEV)
    labels = torch.randint(0, K, (N,), generator=g).to(DEV)
    xm = torch.empty(N, Cf, device=DEV)
    logits = torch.empty(N, K, device=DEV)
    C.head_forward(feat, W, b, p, seed, xm, logits)
    dl = torch.empty(N, K, device=DEV)
    loss = torch.empty(1, device=DEV)
    counts = torch.zeros(2, dtype=torch.long, device=DEV)
    rl = torch.empty(N, device=DEV)
    rc = torch.empty(N, dtype=torch.int32, device=DEV)
    C.head_ce(logits, labels, scale / N, dl, loss, counts, 0, rl, rc)
    gW0 = torch.randn(K, Cf, generator=g).to(DEV)
    gb0 = torch.randn(K, generator=g).to(DEV)
    gW, gb = gW0.clone(), gb0.clone()
    dfeat = torch.empty(N, P, Cf, device=DEV)
    scratch = torch.empty(K * N + Cf * N + Cf * K, device=DEV)
    C.head_backward(dl, xm, W, P, p, seed, gW, gb, beta, dfeat, scratch)
    mask = torch.empty(N, P, Cf, dtype=torch.uint8, device=DEV)
    C.head_dropout_mask(mask, p, seed)
    torch.cuda.synchronize()
    r_logits, r_loss, r_gW, r_gb, r_df = _ref(feat.cpu(), W.cpu(), b.cpu(), labels.cpu(), mask.cpu(), p, scale)
    return dict(logits=(logits, r_logits), loss=(loss[0], r_loss), gW=(gW, r_gW + beta * gW0.cpu().double()),
                gb=(gb, r_gb + beta * gb0.cpu().double()), dfeat=(dfeat, r_df), counts=counts,
                labels=labels, mask=mask)


def _close(a, ref, tol):
    a = a.detach().double().cpu()
    err = (a - ref).norm() / ref.norm().clamp_min(1e-30)
    assert err < tol, float(err)


@pytest.mark.parametrize("N,P,Cf,K", [(5, 4, 40, 7), (16, 1, 2304, 400), (3, 2, 2304, 700), (33, 1, 96, 17)])
def test_head_matches_fp64(N, P, Cf, K):
    r = _run(N, P, Cf, K, p=0.0)
    for k in ("logits", "gW", "gb", "dfeat"):
        _close(r[k][0], r[k][1], 1e-5)
    assert abs(float(r["loss"][0]) - float(r["loss"][1])) < 1e-5 * max(1.0, float(r["loss"][1]))
    preds = r["logits"][0].argmax(-1)
    assert int(r["counts"][0]) == int((preds == r["labels"]).sum()) and int(r["counts"][1]) == N


def test_head_dropout_and_accumulate():
    r = _run(8, 4, 256, 10, p=0.5, beta=1.0)
    keep = r["mask"].float().mean().item()
    assert 0.45 < keep < 0.55            # Bernoulli(0.5) keep rate
    for k in ("logits", "gW", "gb", "dfeat"):
        _close(r[k][0], r[k][1], 1e-5)
    assert torch.all(r["dfeat"][0][r["mask"] == 0] == 0)


def test_head_eval_counts_ties_and_accumulation():
    C = _C()
    logits = torch.tensor([[1.0, 3.0, 3.0], [0.5, 0.1, 0.2], [2.0, 2.0, 2.0]], device=DEV)
    labels = torch.tensor([1, 0, 2], device=DEV)    # ties resolve to the first maximum (torch.argmax)
    counts = torch.zeros(2, dtype=torch.long, device=DEV)
    rl = torch.empty(3, device=DEV)
    rc = torch.empty(3, dtype=torch.int32, device=DEV)
    C.head_ce(logits, labels, 0.0, None, None, counts, 1, rl, rc)
    C.head_ce(logits, labels, 0.0, None, None, counts, 1, rl, rc)
    assert counts.tolist() == [4, 6]
