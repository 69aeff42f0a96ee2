# DP (2 ranks, gloo, one GPU) deterministic gradient vs the mean of single-rank gradients: default buckets vs one
# bucket launched at the end of backward; three repetitions each (numeric check, no fault involved).
import json, os, subprocess, sys, torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "gpurun_out", "dp_det_check")
os.makedirs(OUT, exist_ok=True)
BASE = ["--batch", "4", "--steps", "3", "--warmup", "1", "--deterministic"]
env = dict(os.environ, OMP_NUM_THREADS="2", PVA_DIST_BACKEND="gloo")
for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
    env.pop(k, None)
def run(args, name):
    dump = os.path.join(OUT, name + ".pt")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + BASE + args + ["--dump", dump],
                       stdout=subprocess.DEVNULL, stderr=open(os.path.join(OUT, name + ".err"), "w"), env=env, timeout=300)
    assert r.returncode == 0, name
    return torch.load(dump, weights_only=True)["grad"]
s = [run(["--gpus", "1", "--data-rank", str(r), "--bucket-mb", "8", "--first-bucket-mb", "1"], f"single{r}") for r in range(2)]
ref = (s[0] + s[1]) / 2
for tag, bk in (("default", ["--bucket-mb", "8", "--first-bucket-mb", "1"]), ("onebucket", ["--bucket-mb", "100000", "--first-bucket-mb", "100000"])):
    for i in range(3):
        g = run(["--gpus", "2"] + bk, f"dp_{tag}{i}")
        print(tag, i, "err %.3e" % float((g - ref).norm() / ref.norm()), flush=True)
