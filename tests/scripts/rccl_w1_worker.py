"""One torchrun rank with PVA_FORCE_GRADSYNC=1 (world size 1, RCCL): drives every DistState collective through
ProcessGroupNCCL and prints one JSON line of results (tests/test_rccl_w1_gpu.py)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from pytorchvideo_accelerate_amd.parallel.dist import DistState  # noqa: E402
from pytorchvideo_accelerate_amd.parallel.ddp import GradSync  # noqa: E402


def main():
    st = DistState.from_env()
    assert st.multi and st.backend == "nccl", (st.multi, st.backend)
    dev = st.device
    out = {"backend": st.backend, "world": st.world_size}
    st.barrier()                                   # barrier(device_ids=...)
    x = torch.arange(12, dtype=torch.float32, device=dev).view(3, 4)
    g = st.all_gather_cat(x)                       # all_gather_into_tensor
    out["gather_ok"] = bool(torch.equal(g, x))
    a = torch.randn(1000, device=dev)
    b = a.clone()
    st.all_reduce_(b, "avg")                       # ReduceOp.AVG
    out["avg_ok"] = bool(torch.equal(a, b))
    out["bcast_obj"] = st.broadcast_object({"k": 3})
    out["agree"] = st.agree_times([1.5, 2.5])
    p = torch.randn(77, device=dev)
    q = p.clone()
    st.broadcast_tensors([q])
    out["bcast_ok"] = bool(torch.equal(p, q))
    # GradSync with per-bucket timing on its comm stream, producers = the current stream
    grad = torch.randn(3 << 20, device=dev)
    ref = grad.clone()
    sync = GradSync(grad, st, bucket_mb=4, first_mb=1, timing=True)
    sync.producers = lambda: [torch.cuda.current_stream(dev)]
    for _ in range(3):
        sync.begin(True)
        sync.progress(grad.numel() // 2)
        sync.finish()
    torch.cuda.synchronize()
    out["sync_ok"] = bool(torch.equal(grad, ref))
    out["stats"] = sync.stats()
    st.destroy()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
