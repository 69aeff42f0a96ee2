"""Diagnostic: per-parameter gradient error of the fused executor with and without BN folding on the
lateral-fusion block test (tests/test_blocks_gpu.py::test_fusion_pathways), vs fp32 oracle and autocast."""
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from pytorchvideo_accelerate_amd.models import reference as R   # noqa: E402
from pytorchvideo_accelerate_amd.models.fused import FusedNet    # noqa: E402
from pytorchvideo_accelerate_amd.ops.conv import Act             # noqa: E402

DEV = torch.device("cuda")


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def build():
    torch.manual_seed(0)
    N, T, H = 2, 8, 8
    blk = R.MultiPathWayWithFuse([R.ResStage(1, 16, 8, 32, 1, 1), R.ResStage(1, 8, 8, 16, 3, 1)],
                                 R.FuseFastToSlow(16, 2, 7, 4))
    R.init_net_weights(blk)
    blk2 = R.MultiPathWayWithFuse([R.ResStage(1, 64, 16, 64, 1, 1), R.ResStage(1, 16, 8, 16, 3, 1)], None)
    R.init_net_weights(blk2)
    pool = R.PoolConcatPathway(((T // 4, H, H), (T, H, H)))
    net = R.Net([blk, blk2, pool, R.create_res_basic_head(80, 10, pool=None, dropout_rate=0.0)])

    def _x(N, C, T, H, W, seed):
        g = torch.Generator().manual_seed(seed)
        return torch.randn(N, C, T, H, W, generator=g).to(torch.bfloat16).float().to(DEV)
    xs = [_x(N, 16, T // 4, H, H, 2), _x(N, 8, T, H, H, 3)]
    return net, xs, torch.arange(N, device=DEV) % 10


def main():
    res = {}
    for fold in ("100000", "8"):
        os.environ["PVA_BN_FOLD_MIN_C"] = fold
        net, xs, labels = build()
        oracle = copy.deepcopy(net).to(DEV).train()
        F.cross_entropy(oracle(xs), labels).backward()
        eng = FusedNet(net, DEV)
        eng.tuner.enabled = os.environ.get("DIAG_TUNE", "1") == "1"
        loss, _ = eng.forward_backward([Act.from_ncthw(x) for x in xs], labels)
        torch.cuda.synchronize()
        ref = dict(oracle.named_parameters())
        res[fold] = {n: (p.grad.clone(), ref[n].grad) for n, p in net.named_parameters()}
        print("fold_min_c", fold, "loss", loss.item(), flush=True)
    for n in res["8"]:
        g1, r = res["100000"][n]
        g2, _ = res["8"][n]
        print("%-70s nofold %.4f fold %.4f fold-vs-nofold %.4f" % (n, rel(g1, r), rel(g2, r), rel(g2, g1)))


if __name__ == "__main__":
    main()
