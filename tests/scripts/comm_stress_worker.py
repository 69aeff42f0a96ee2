"""Comm-overlap stress test worker (SURVEY.md §5 race detection): GradSync under random timing.

Each rank "runs backward" by writing the flat gradient in random-size chunks with random delays and
reporting progress at random points, so buckets are launched at different moments on different ranks;
mixes no_sync micro-steps (accumulation) and a restricted span.  Every result is checked exactly."""
import json
import os
import random
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorchvideo_accelerate_amd.parallel.ddp import GradSync  # noqa: E402
from pytorchvideo_accelerate_amd.parallel.dist import DistState  # noqa: E402


def backward(grad, sync, rng, values):
    n = grad.numel()
    off = 0
    while off < n:
        step = rng.randint(1, max(1, n // 7))
        hi = min(n, off + step)
        grad[off:hi] += values[off:hi]
        off = hi
        if rng.random() < 0.3:
            time.sleep(rng.random() * 0.004)
        if rng.random() < 0.7:
            sync.progress(off if rng.random() < 0.8 else rng.randint(0, off))  # stale reports allowed


def main():
    out = sys.argv[1]
    st = DistState.from_env(cpu=True)
    W, r = st.world_size, st.rank
    rng = random.Random(1000 + r)
    n = 50_000
    bounds = sorted(random.Random(7).sample(range(1, n), 60)) + [n]
    grad = torch.zeros(n, dtype=torch.float64)
    sync = GradSync(grad, st, bucket_mb=0.02, boundaries=bounds)
    errs = []
    for it in range(30):
        micro = 1 + it % 3
        grad.zero_()
        for m in range(micro):
            vals = [torch.arange(n, dtype=torch.float64) * (k + 1) + 1000 * it + 10 * m for k in range(W)]
            sync.begin(m == micro - 1)          # no_sync on all but the last micro-step
            backward(grad, sync, rng, vals[r])
            sync.finish()
        # the no_sync steps accumulate locally; the final synced all-reduce averages the accumulation
        full = torch.zeros(n, dtype=torch.float64)
        for m in range(micro):
            full += sum(torch.arange(n, dtype=torch.float64) * (k + 1) + 1000 * it + 10 * m for k in range(W)) / W
        errs.append(float((grad - full).abs().max()))
    # restricted span: only [lo, hi) is averaged, the rest stays local
    lo, hi = bounds[10], bounds[40]
    sync2 = GradSync(grad, st, bucket_mb=0.02, boundaries=bounds)
    sync2.restrict(lo, hi)
    grad.fill_(float(r + 1))
    sync2.begin(True)
    backward(grad, sync2, rng, torch.zeros(n, dtype=torch.float64))
    sync2.finish()
    mean = sum(range(1, W + 1)) / W
    ok_span = bool((grad[lo:hi] == mean).all()) and bool((grad[:lo] == r + 1).all()) and bool((grad[hi:] == r + 1).all())
    if r == 0:
        json.dump({"max_err": max(errs), "ok_span": ok_span, "buckets": len(sync.buckets)}, open(out, "w"))
    st.destroy()


if __name__ == "__main__":
    main()
