"""Gradient error spread of the noise-dominated lateral-fusion block test (tests/test_blocks_gpu.py::
test_fusion_pathways) under kernel-selection knobs: per parameter rel-L2 vs the fp32 oracle for each setting.
python scripts/diag_fusion_noise.py"""
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchvideo_accelerate_amd.models import reference as R  # noqa: E402
from pytorchvideo_accelerate_amd.models.fused import FusedNet  # noqa: E402
from pytorchvideo_accelerate_amd.ops.conv import Act  # noqa: E402

DEV = torch.device("cuda")


def _x(N, C, T, H, W, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(N, C, T, H, W, generator=g).to(torch.bfloat16).float().to(DEV)


def _act(x):
    return Act.from_ncthw(x)


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def main():
    os.environ["PVA_BN_FOLD_MIN_C"] = "100000"
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
    oracle = copy.deepcopy(net).to(DEV).train()
    F.cross_entropy(oracle(xs), labels).backward()
    ref = dict(oracle.named_parameters())
    m = copy.deepcopy(net).to(DEV).train()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = m(xs)
    F.cross_entropy(out.float(), labels).backward()
    ac = {n: rel(p.grad, ref[n].grad) for n, p in m.named_parameters()}
    names = [n for n in ac if "norm_a" in n or "norm_b" in n][:6]
    print("autocast    " + " ".join(f"{ac[n]:.3f}" for n in names), flush=True)
    for knobs in ({"PVA_CONV_PW_W4": "0"}, {"PVA_CONV_PW_W4": "1"}, {"PVA_CONV_PW": "0"}, {"PVA_AUTOTUNE": "0"},
                  {"PVA_CONV_PW_W4": "1"}, {"PVA_CONV_PW_W4": "0"}):
        saved = {k: os.environ.get(k) for k in knobs}
        os.environ.update(knobs)
        os.environ["PVA_TUNE_CACHE"] = "0"
        n1 = copy.deepcopy(net)
        eng = FusedNet(n1, DEV)
        eng.forward_backward([_act(x) for x in xs], labels)
        torch.cuda.synchronize()
        e = {n: rel(p.grad, ref[n].grad) for n, p in n1.named_parameters()}
        print(f"{str(knobs):28s} " + " ".join(f"{e[n]:.3f}" for n in names), flush=True)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    print("params: " + ", ".join(names))


if __name__ == "__main__":
    main()
