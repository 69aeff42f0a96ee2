"""Small-batch training trajectory: B=16 SlowFast-R50 32x2x224, lr 0.1, momentum 0.9,
wd 1e-4, fresh random clips and labels every step, from identical weights -- the fused executor vs the PyTorch
modules in fp32 and under bf16 autocast (the reference recipe, run.py:253-261).  Dropout is off in all three
(the masks could not match).  Prints the three loss trajectories and the max |log-ratio| of the weight norms."""
import copy
import json
import os
import sys

import torch
import torch.nn.functional as F

os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def clips(B, step, alpha=4):
    g = torch.Generator().manual_seed(100 + step)
    fast = torch.randn(B, 3, 32, 224, 224, generator=g).to(torch.bfloat16).float()
    labels = torch.randint(0, 400, (B,), generator=g)
    return [fast[:, :, ::alpha].contiguous(), fast], labels


def main():
    from pytorchvideo_accelerate_amd.models import reference as R
    from pytorchvideo_accelerate_amd.models.fused import FusedNet
    from pytorchvideo_accelerate_amd.ops.optim import FusedSGD
    B = int(os.environ.get("B", "16"))
    steps = int(os.environ.get("STEPS", "10"))
    lr = float(os.environ.get("LR", "0.1"))
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = R.create_slowfast(50, 400, dropout_rate=0.0)
    init = copy.deepcopy(model)
    res = {}
    for mode in ("fp32", "autocast"):
        m = copy.deepcopy(init).to(dev).train()
        opt = torch.optim.SGD(m.parameters(), lr=lr, momentum=0.9, weight_decay=1e-4)
        ls = []
        for s in range(steps):
            xs, y = clips(B, s)
            opt.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=mode == "autocast"):
                out = m([x.to(dev) for x in xs])
            loss = F.cross_entropy(out.float(), y.to(dev))
            loss.backward()
            opt.step()
            ls.append(round(float(loss), 4))
        res[mode] = ls
        print(mode, ls, flush=True)
        del m, opt
        torch.cuda.empty_cache()
    eng = FusedNet(model, dev)
    opt = FusedSGD(eng.flat, lr=lr, momentum=0.9, weight_decay=1e-4, after_step=eng.pack)
    ls = []
    for s in range(steps):
        xs, y = clips(B, s)
        opt.zero_grad()
        loss, _ = eng.forward_backward(eng.prepare_inputs(xs), y.to(dev))
        opt.step()
        ls.append(round(float(loss), 4))
    res["fused"] = ls
    print("fused", ls, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
