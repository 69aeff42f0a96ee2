"""Run-to-run reproducibility of the single-process production schedule (two streams, heuristic kernels) with the
lateral-fusion backward on either stream (PVA_SIDE_FUSE=1 / 0): two identical bench.py runs on the same data shard
must give the same flat gradient up to the fp32-atomic noise of the leaf weight gradients (tests/test_dp_fused_gpu.py
relies on it).  Prints one line per setting: the relative difference between the two runs."""
import os
import subprocess
import sys
import tempfile

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--batch", "4", "--steps", "3", "--warmup", "1", "--gpus", "1", "--data-rank", "0"]


def run(tmp, name, **env):
    dump = os.path.join(tmp, name + ".pt")
    e = dict(os.environ, PVA_AUTOTUNE="0", **env)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + ARGS + ["--dump", dump],
                       capture_output=True, text=True, timeout=400, env=e)
    assert r.returncode == 0, r.stderr[-3000:]
    return torch.load(dump, weights_only=True)["grad"]


def main():
    with tempfile.TemporaryDirectory() as tmp:
        for flag in sys.argv[1:] or ["0", "1"]:
            a = run(tmp, f"a{flag}", PVA_SIDE_FUSE=flag)
            b = run(tmp, f"b{flag}", PVA_SIDE_FUSE=flag)
            print(f"PVA_SIDE_FUSE={flag}: run-to-run rel diff {float((a - b).norm() / a.norm()):.3e}", flush=True)


if __name__ == "__main__":
    main()
