"""Narrow fused backward / narrow fold vs the unfused path and the fp32 oracle: per-parameter gradient rel-L2 of each
variant (the worst parameters named) at a small SlowFast shape.  python scripts/diag_narrow.py"""
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchvideo_accelerate_amd.models import reference as R  # noqa: E402
from pytorchvideo_accelerate_amd.models.fused import FusedNet  # noqa: E402

DEV = torch.device("cuda")


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def main():
    torch.manual_seed(0)
    model = R.create_slowfast(50, 10, head_pool_kernel_sizes=((4, 3, 3), (16, 3, 3)), dropout_rate=0.0)
    g = torch.Generator().manual_seed(3)
    fast = torch.randn(2, 3, 16, 96, 96, generator=g).to(torch.bfloat16).float()
    xs = [fast[:, :, torch.linspace(0, 15, 4).long()].contiguous(), fast]
    labels = torch.tensor([2, 5], device=DEV)
    oracle = copy.deepcopy(model).to(DEV).train()
    F.cross_entropy(oracle([x.to(DEV) for x in xs]), labels).backward()
    ref = {n: p.grad for n, p in oracle.named_parameters()}
    res = {}
    for det in (True, False):
        for flag, fold in (("1", "1"), ("1", "0"), ("0", "0")):
            os.environ["PVA_NARROW_BWD"], os.environ["PVA_NARROW_FOLD"] = flag, fold
            m = copy.deepcopy(model)
            eng = FusedNet(m, DEV, deterministic=det)
            loss, _ = eng.forward_backward(eng.prepare_inputs(xs), labels)
            torch.cuda.synchronize()
            gr = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
            res[(det, flag, fold)] = gr
            errs = sorted(((rel(gr[n], ref[n]), n) for n in ref if ref[n].norm() > 0), reverse=True)
            print(f"det={det} narrow={flag} fold={fold} loss={float(loss):.5f} median-vs-oracle "
                  f"{errs[len(errs) // 2][0]:.4f} worst: " + ", ".join(f"{n} {e:.3f}" for e, n in errs[:5]),
                  flush=True)
        base = res[(det, "0", "0")]
        for key in ((det, "1", "1"), (det, "1", "0")):
            errs = sorted(((rel(res[key][n], base[n]), n) for n in base if base[n].norm() > 0), reverse=True)
            print(f"  {key} vs unfused: median {errs[len(errs) // 2][0]:.4f} worst: "
                  + ", ".join(f"{n} {e:.3f}" for e, n in errs[:8]), flush=True)


if __name__ == "__main__":
    main()
