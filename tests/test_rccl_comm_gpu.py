"""Framework-owned RCCL communicator (csrc/runtime/rccl_comm.cpp, parallel/rccl.py) at world size 1
on the test box's GPU: every collective against its single-rank identity (sum / avg / max all-reduce, broadcast,
all-gather, reduce-scatter; fp32 / bf16 / int64), stream ordering through the returned event, and the library bound
being torch's own RCCL (one copy in the process)."""
import torch

import pytest

pytestmark = pytest.mark.gpu


def test_rccl_communicator_single_rank_collectives():
    from pytorchvideo_accelerate_amd.parallel.rccl import RcclCommunicator
    torch.cuda.set_device(0)
    comm = RcclCommunicator(0, 1)
    assert comm.version >= 21000 and comm.device == 0
    for dt in (torch.float32, torch.bfloat16, torch.int64):
        x = (torch.arange(4099, device="cuda") % 97).to(dt)
        for op in ("sum", "max", "min") + (("avg",) if dt.is_floating_point else ()):
            y = x.clone()
            comm.all_reduce_(y, op).wait()
            assert torch.equal(y, x), (dt, op)
        y = x.clone()
        comm.broadcast_(y, 0).wait()
        assert torch.equal(y, x)
        out = torch.empty_like(x)
        comm.all_gather(out, x).wait()
        assert torch.equal(out, x)
        out = torch.empty_like(x)
        comm.reduce_scatter(out, x, "sum").wait()
        assert torch.equal(out, x)
    # ordering: a collective enqueued on a side stream, the current stream waits on its event
    side = torch.cuda.Stream()
    z = torch.full((1 << 20,), 2.0, device="cuda")
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        w = comm.all_reduce_(z, "sum")
    w.wait()
    z.mul_(3.0)
    assert float(z[0]) == 6.0 and float(z[-1]) == 6.0
    comm.close()


def test_rccl_bound_to_torch_copy():
    import os
    from pytorchvideo_accelerate_amd.parallel.rccl import torch_rccl_path
    from pytorchvideo_accelerate_amd.parallel.rccl import RcclCommunicator
    RcclCommunicator(0, 1).close()
    maps = open(f"/proc/{os.getpid()}/maps").read()
    libs = {line.split()[-1] for line in maps.splitlines() if "librccl" in line}
    assert len(libs) == 1 and os.path.realpath(torch_rccl_path()) in {os.path.realpath(p) for p in libs}, libs
