"""Multi-process data parallel on CPU (gloo, world size 2) — SURVEY.md §4.3 item 4."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(args, nproc=2, timeout=600, cwd=None):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}"] + args
    env = dict(os.environ, OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=cwd or REPO, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r


def test_gradsync_equals_big_batch(tmp_path):
    out = str(tmp_path / "res.json")
    _launch([os.path.join(HERE, "scripts", "ddp_worker.py"), out])
    res = json.load(open(out))
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(6, 16), torch.nn.Tanh(), torch.nn.Linear(16, 3))
    g = torch.Generator().manual_seed(123)
    X = torch.randn(8, 6, generator=g)
    Y = torch.randint(0, 3, (8,), generator=g)
    torch.nn.functional.cross_entropy(net(X), Y).backward()
    ref = torch.cat([p.grad.reshape(-1) for p in reversed(list(net.parameters()))])
    got = torch.tensor(res["grad"])
    # flat buffer pads every tensor to a multiple of 4 elements; compare per tensor
    off, chunks = 0, []
    for p in reversed(list(net.parameters())):
        chunks.append(got[off:off + p.numel()])
        off += (p.numel() + 3) // 4 * 4
    torch.testing.assert_close(torch.cat(chunks), ref, rtol=1e-5, atol=1e-6)
    acc = torch.tensor(res["accum_grad"])
    chunks = []
    off = 0
    for p in reversed(list(net.parameters())):
        chunks.append(acc[off:off + p.numel()])
        off += (p.numel() + 3) // 4 * 4
    torch.testing.assert_close(torch.cat(chunks), ref, rtol=1e-5, atol=1e-6)  # no_sync accumulation
    assert res["params_equal"] and res["avg"] == 1.5 and res["gather"] == [0, 1]


def test_gradsync_stress_random_timing(tmp_path):
    """3 ranks, random chunked backward with random delays / stale progress reports, no_sync accumulation,
    restricted span: the all-reduced gradients are exact (float64 payload)."""
    out = str(tmp_path / "stress.json")
    _launch([os.path.join(HERE, "scripts", "comm_stress_worker.py"), out], nproc=3)
    res = json.load(open(out))
    assert res["max_err"] == 0.0 and res["ok_span"] and res["buckets"] >= 10


@pytest.mark.slow
def test_run_py_two_ranks_cpu(tmp_path):
    args = [os.path.join(REPO, "run.py"), "--cpu", "--synthetic", "--synthetic_videos", "8", "--synthetic_classes",
            "3", "--is_slowfast", "--num_frames", "8", "--crop_size", "64", "--batch_size", "2", "--num_workers",
            "0", "--num_epochs", "1", "--limit_train_batches", "1", "--limit_val_batches", "0",
            "--checkpointing_steps", "2", "--output_dir", str(tmp_path / "out"), "--gradient_accumulation_steps", "2",
            "--quiet"]
    _launch(args, cwd=str(tmp_path))
    d = tmp_path / "out" / "step_2"
    assert (d / "model.safetensors").exists() and (d / "random_states_0.pkl").exists()
    assert (d / "random_states_1.pkl").exists()
    assert (tmp_path / "out" / "final" / "optimizer.bin").exists() or (d / "optimizer.bin").exists()


def test_torch_backend_overlaps_allreduce_with_backward():
    """The PyTorch-module path (``--mixed_precision no`` / CPU) launches gradient buckets from autograd hooks while
    backward runs (DDP-style overlap), front to back over the flat buffer, before ``finish``."""
    import torch
    from pytorchvideo_accelerate_amd.engine.backends import TorchBackend
    from pytorchvideo_accelerate_amd.models import reference as R
    from pytorchvideo_accelerate_amd.parallel.dist import DistState

    torch.manual_seed(0)
    model = R.create_slowfast(50, 5, dropout_rate=0.0, head_pool_kernel_sizes=((2, 2, 2), (8, 2, 2)))
    be = TorchBackend(model, DistState(), "no")

    class Rec:
        active = False

        def __init__(self):
            self.calls, self.finished_after = [], None

        def begin(self, sync=True):
            self.active = sync

        def progress(self, off):
            self.calls.append(off)

        def finish(self):
            self.finished_after = len(self.calls)
            self.active = False

    rec = Rec()
    be.sync = rec
    be.train()
    fast = torch.randn(2, 3, 8, 64, 64)
    xs = [fast[:, :, ::4].contiguous(), fast]
    be.train_step(xs, torch.tensor([1, 3]))
    assert len(rec.calls) > 10, rec.calls
    assert rec.calls == sorted(rec.calls) and rec.calls[-1] == be.flat.span(be.flat.params[-1])[1]
    assert rec.finished_after == len(rec.calls)
    # every bucket end is reached before finish(): nothing left for the end-of-backward flush
    rec2 = Rec()
    be.sync = rec2
    be.train_step(xs, torch.tensor([0, 2]), sync=False)
    assert rec2.calls == []
