"""The RCCL code paths at world size 1.  ``PVA_FORCE_GRADSYNC=1`` makes a
single torchrun rank initialise ProcessGroupNCCL and run every collective — ``ReduceOp.AVG``, the framework's
event-gated comm stream and per-bucket timing (``parallel/ddp.py``), ``barrier(device_ids)``,
``all_gather_into_tensor``, ``broadcast_object`` — on the one GPU of the test box.  The all-reduced gradient of a
deterministic fused step must equal the un-synced run bit for bit (AVG over one rank)."""
import json
import math
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)

BENCH = ["--gpus", "1", "--batch", "4", "--steps", "2", "--warmup", "1", "--bucket-mb", "8",
         "--first-bucket-mb", "1", "--deterministic"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(**kw):
    env = dict(os.environ, OMP_NUM_THREADS="2", **kw)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "PVA_DIST_BACKEND"):
        env.pop(k, None)
    return env


def _torchrun(script_args, tmp_path, **env):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_port()}"] + script_args
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, cwd=str(tmp_path),
                       env=_env(PVA_FORCE_GRADSYNC="1", **env))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_rccl_collectives_world_size_one(tmp_path):
    out = _torchrun([os.path.join(HERE, "scripts", "rccl_w1_worker.py")], tmp_path)
    assert out["backend"] == "nccl" and out["world"] == 1
    assert out["gather_ok"] and out["avg_ok"] and out["bcast_ok"] and out["sync_ok"]
    assert out["bcast_obj"] == {"k": 3} and out["agree"] == [1.5, 2.5]
    st = out["stats"]
    assert st["buckets"] >= 3
    for k in ("comm_exposed_ms", "comm_bucket_ms", "comm_last_bucket_ms"):
        assert math.isfinite(st[k]) and st[k] >= 0, st


@pytest.mark.parametrize("comm", ["pg", "rccl"])
def test_rccl_forced_gradsync_bench_matches_unsynced(tmp_path, comm):
    """``comm``: the bucket all-reduce through ProcessGroupNCCL, or through the framework-owned communicator
    (``PVA_COMM=rccl``, parallel/rccl.py)."""
    d1 = str(tmp_path / "rccl.pt")
    res = _torchrun([os.path.join(REPO, "bench.py")] + BENCH + ["--dump", d1], tmp_path, PVA_COMM=comm)
    cfg = res["config"]
    assert cfg["backend"] == "nccl" and cfg["forced_sync"] is True and res["n_gpus"] == 1
    assert cfg["comm"] == ("framework-rccl" if comm == "rccl" else "process-group"), cfg["comm"]
    for k in ("comm_exposed_ms", "comm_bucket_ms", "comm_last_bucket_ms"):
        assert k in cfg and math.isfinite(cfg[k]), cfg
    assert cfg["buckets"] > 1
    d0 = str(tmp_path / "plain.pt")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + BENCH + ["--dump", d0],
                       capture_output=True, text=True, timeout=400, cwd=str(tmp_path), env=_env())
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    g1 = torch.load(d1, weights_only=True)["grad"]
    g0 = torch.load(d0, weights_only=True)["grad"]
    assert torch.equal(g0, g1), float((g0 - g1).abs().max())
