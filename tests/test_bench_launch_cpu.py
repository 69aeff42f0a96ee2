"""bench.py's multi-rank self-launch path (``--gpus N`` → child torchrun → N ranks), rehearsed on CPU/gloo
with ``--plumbing``: the JSON line reports the whole job, every rank ends with identical weights and the
all-reduced gradient equals the mean of the per-rank gradients (DDP semantics, per-rank BN statistics)."""
import json
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)

ARGS = ["--plumbing", "--steps", "1", "--warmup", "1", "--batch", "2", "--frames", "8", "--crop", "64",
        "--classes", "5", "--bucket-mb", "8", "--first-bucket-mb", "1"]


def _run(extra, tmp_path):
    env = dict(os.environ, OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + ARGS + extra, capture_output=True,
                       text=True, timeout=900, cwd=str(tmp_path), env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_self_launch_two_ranks(tmp_path):
    dump = str(tmp_path / "dump.pt")
    res = _run(["--gpus", "2", "--dump", dump], tmp_path)
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2"
    assert res["config"]["global_batch"] == 4 and res["value"] > 0 and res["steps"] == 1
    d = torch.load(dump, weights_only=True)
    assert d["world_size"] == 2
    torch.testing.assert_close(d["params"][0], d["params"][1], rtol=0, atol=0)

    import bench
    from pytorchvideo_accelerate_amd.engine.backends import TorchBackend
    from pytorchvideo_accelerate_amd.parallel.dist import DistState

    a = bench.parse(ARGS)
    be = TorchBackend(bench.plumbing_model(a), DistState(), "no")
    be.train()
    for r in range(2):   # mean over ranks of per-rank gradients (each rank its own BN batch statistics)
        xs, y = bench.plumbing_batch(a, r, 0)
        be.train_step(xs, y, loss_scale=0.5)
    ref = be.flat.grad
    got = d["grad"]
    assert got.shape == ref.shape
    err = (got - ref).norm() / ref.norm()
    assert err < 1e-5, float(err)


def test_bench_single_rank_plumbing(tmp_path):
    res = _run(["--gpus", "1"], tmp_path)
    assert res["n_gpus"] == 1 and res["config"]["parallelism"] == "dp1"


def test_forced_gradsync_single_rank_gloo(tmp_path):
    """``PVA_FORCE_GRADSYNC=1`` at world size 1: a real (gloo) process group, every bucket all-reduced through it;
    the gradient equals the un-synced single-process run bit for bit (average over one rank)."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
               PVA_FORCE_GRADSYNC="1")
    env.pop("WORLD_SIZE", None)
    d1 = str(tmp_path / "forced.pt")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                        "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(REPO, "bench.py"),
                        "--gpus", "1", "--dump", d1] + ARGS, capture_output=True, text=True, timeout=900,
                       cwd=str(tmp_path), env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert res["config"]["backend"] == "gloo" and res["config"]["forced_sync"] is True
    d0 = str(tmp_path / "plain.pt")
    res0 = _run(["--gpus", "1", "--dump", d0], tmp_path)
    assert res0["config"]["backend"] == "none"
    g1 = torch.load(d1, weights_only=True)["grad"]
    g0 = torch.load(d0, weights_only=True)["grad"]
    assert torch.equal(g0, g1)
