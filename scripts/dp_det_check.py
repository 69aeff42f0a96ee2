"""DP (2 gloo ranks sharing one GPU) deterministic gradient vs the mean of single-rank gradients, repeated, optionally
under a concurrent GPU load (``--load``): prints the relative error and, when non-zero, where in the flat gradient
the differences sit (a race on an all-reduce bucket stays inside that bucket's range; a perturbed computation spreads
over every parameter whose gradient is computed after it).  Numeric check only — no fault is involved."""
import argparse, os, subprocess, sys, torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "gpurun_out", "dp_det_check")
os.makedirs(OUT, exist_ok=True)
ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--load", action="store_true")
ap.add_argument("--single-load", action="store_true", help="repeat single-rank 0 under the load instead of DP runs")
a = ap.parse_args()
BASE = ["--batch", "4", "--steps", "3", "--warmup", "1", "--deterministic", "--bucket-mb", "8", "--first-bucket-mb", "1"]
env = dict(os.environ, OMP_NUM_THREADS="2", PVA_DIST_BACKEND="gloo")
for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
    env.pop(k, None)
def run(args, name):
    dump = os.path.join(OUT, name + ".pt")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + BASE + args + ["--dump", dump],
                       stdout=subprocess.DEVNULL, stderr=open(os.path.join(OUT, name + ".err"), "w"), env=env, timeout=300)
    assert r.returncode == 0, name
    g = torch.load(dump, weights_only=True)["grad"]
    os.remove(dump)
    return g
s = [run(["--gpus", "1", "--data-rank", str(r)], f"single{r}") for r in range(2)]
ref = (s[0] + s[1]) / 2
load = None
if a.load:
    load = subprocess.Popen(["timeout", "-k", "10", "400", sys.executable, os.path.join(REPO, "bench.py"), "--batch", "32",
                             "--steps", "2000", "--warmup", "1"], stdout=subprocess.DEVNULL,
                            stderr=open(os.path.join(OUT, "load.err"), "w"))
try:
    for i in range(a.reps):
        g = run(["--gpus", "1", "--data-rank", "0"], f"s0_{i}") if a.single_load else run(["--gpus", "2"], f"dp{i}")
        if a.single_load:
            ref = s[0]   # same rank, same data: any difference is run-to-run noise under the load
        d = (g - ref).abs()
        nz = (d > 0).nonzero().flatten()
        msg = "err %.3e" % float((g - ref).norm() / ref.norm())
        if nz.numel():
            msg += " differing %d of %d, flat index %d..%d (numel %d)" % (nz.numel(), d.numel(), int(nz[0]), int(nz[-1]), d.numel())
        print("rep", i, msg, flush=True)
finally:
    if load is not None:
        load.kill(); load.wait()
