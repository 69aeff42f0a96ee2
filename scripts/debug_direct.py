"""Locate the first conv whose output differs between the direct kernel and the implicit-GEMM kernel.

    python scripts/debug_direct.py
Runs the fused SlowFast forward+backward of tests/test_fused_gpu.py twice on identical copies of the model:
once with PVA_CONV_DIRECT=0 (implicit GEMM only), once forcing the direct kernel wherever it is legal,
and prints per-workspace relative differences in execution order."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--force", default="512", choices=["512", "2k", "tuned"],
                    help="direct run: force the 512-row / 2048-row direct kernel, or let the tuner choose")
    a = ap.parse_args()
    S, B = a.size, a.batch
    f = S // 32
    from pytorchvideo_accelerate_amd.models import reference as R
    from pytorchvideo_accelerate_amd.models.fused import FusedNet
    from pytorchvideo_accelerate_amd.ops import tune
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = R.create_slowfast(50, 10, head_pool_kernel_sizes=((2, f, f), (8, f, f)), dropout_rate=0.0)
    g = torch.Generator().manual_seed(0)
    fast = torch.randn(B, 3, 8, S, S, generator=g).to(torch.bfloat16).float()
    idx = torch.linspace(0, 7, 2).long()
    xs = [fast[:, :, idx].contiguous(), fast]
    labels = torch.arange(B, device=dev) % 10
    res = {}
    for mode in ("igemm", "direct"):
        m = copy.deepcopy(model)
        eng = FusedNet(m, dev)
        if mode == "igemm":
            eng.tuner.direct = False
            eng.tuner.enabled = False
        else:
            orig = eng.tuner.candidates

            def only_direct(gg, chunk, orig=orig):
                c = orig(gg, chunk)
                want = tune.DIRECT_2K if a.force == "2k" else 0
                d = [x for x in c if x & tune.DIRECT and (x & tune.DIRECT_2K) == want]
                return d or c
            if a.force != "tuned":
                eng.tuner.candidates = only_direct
            eng.tuner.log = True
        loss, _ = eng.forward_backward(eng.prepare_inputs(xs), labels)
        torch.cuda.synchronize()
        res[mode] = (float(loss), {k: v.clone() for k, v in eng._ws.items()}, eng.flat.grad.clone())
        print(mode, "loss", float(loss))
    a, b = res["igemm"][1], res["direct"][1]
    for k in a:
        if k in b and a[k].dtype in (torch.bfloat16, torch.float32):
            x, y = a[k].float(), b[k].float()
            r = ((x - y).norm() / x.norm().clamp_min(1e-12)).item()
            flag = " <<<" if r > 2e-2 else ""
            if "stats" not in str(k):
                print(f"{str(k):60s} {r:.3e}{flag}")
    ga, gb = res["igemm"][2], res["direct"][2]
    print("grad rel", ((ga - gb).norm() / ga.norm()).item())


if __name__ == "__main__":
    main()
