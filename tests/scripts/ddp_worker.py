"""Worker for tests/test_ddp_cpu.py (launched by torch.distributed.run, gloo backend)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorchvideo_accelerate_amd.models.fused import FlatParams  # noqa: E402
from pytorchvideo_accelerate_amd.ops.optim import FusedSGD  # noqa: E402
from pytorchvideo_accelerate_amd.parallel.ddp import GradSync  # noqa: E402
from pytorchvideo_accelerate_amd.parallel.dist import DistState  # noqa: E402


def main():
    out = sys.argv[1]
    st = DistState.from_env(cpu=True)
    assert st.backend == "gloo" and st.world_size == 2
    torch.manual_seed(0)  # identical init everywhere, then broadcast anyway
    net = torch.nn.Sequential(torch.nn.Linear(6, 16), torch.nn.Tanh(), torch.nn.Linear(16, 3))
    flat = FlatParams(list(reversed(list(net.named_parameters()))), torch.device("cpu"))
    st.broadcast_tensors([flat.data])
    sync = GradSync(flat.grad, st, bucket_mb=0.0001)  # many tiny buckets
    opt = FusedSGD(flat, lr=0.1, momentum=0.9, weight_decay=1e-4, params=list(net.parameters()))
    g = torch.Generator().manual_seed(123)
    X = torch.randn(8, 6, generator=g)
    Y = torch.randint(0, 3, (8,), generator=g)
    res = {}
    # (1) one synced step on the rank's half == big-batch gradient on one process
    xs, ys = X[st.rank * 4:(st.rank + 1) * 4], Y[st.rank * 4:(st.rank + 1) * 4]
    flat.grad.zero_()
    loss = torch.nn.functional.cross_entropy(net(xs), ys)
    loss.backward()
    flat.rebind()
    sync.begin(True)
    sync.progress(flat.numel // 2)
    sync.finish()
    res["grad"] = flat.grad.tolist()
    # (2) gradient accumulation with no_sync on the first micro-step
    flat.grad.zero_()
    for k, do_sync in ((0, False), (1, True)):
        xb = X[st.rank * 4 + 2 * k: st.rank * 4 + 2 * k + 2]
        yb = Y[st.rank * 4 + 2 * k: st.rank * 4 + 2 * k + 2]
        (torch.nn.functional.cross_entropy(net(xb), yb) / 2).backward()
        flat.rebind()
        sync.begin(do_sync)
        sync.finish()
    res["accum_grad"] = flat.grad.tolist()
    opt.step()
    params = flat.data.clone()
    gathered = st.all_gather_cat(params.unsqueeze(0))
    res["params_equal"] = bool(torch.equal(gathered[0], gathered[1]))
    t = torch.tensor([st.rank + 1.0])
    st.all_reduce_(t, "avg")
    res["avg"] = t.item()
    g2 = st.all_gather_cat(torch.tensor([st.rank]))
    res["gather"] = g2.tolist()
    if st.rank == 0:
        with open(out, "w") as fh:
            json.dump(res, fh)
    st.destroy()


if __name__ == "__main__":
    main()
