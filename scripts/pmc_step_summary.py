"""Per-kernel PMC summary of ONE steady-state training step of bench.py (rocprofv3 --pmc passes).

Each pass directory holds a ``*counter_collection.csv``; dispatches are kept only between the last two
``sgd_momentum_kernel`` dispatches (one optimizer step, after autotuning), then summed per kernel
instantiation and reported with derived ratios:

  mfma%   = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE)         matrix-pipe busy share of the kernel's time
  valu/mf = SQ_INSTS_VALU / SQ_INSTS_MFMA
  wait    = SQ_WAIT_ANY / SQ_WAVE_CYCLES  (parked on s_waitcnt / barrier)
  lds_cf  = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  GB      = 2 * FETCH_SIZE (gfx950 FETCH_SIZE reports half of wide streaming reads) and WRITE_SIZE
  l2hit   = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)   (when that pass was collected)

    python scripts/pmc_step_summary.py gpurun_out/pmc_step > profiles/.../pmc_step.txt
"""
import collections
import csv
import glob
import os
import sys


def load_pass(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return {}, {}
    rows = list(csv.DictReader(open(f[0])))
    by_disp = collections.defaultdict(dict)
    meta = {}
    for r in rows:
        did = int(r["Dispatch_Id"])
        by_disp[did][r["Counter_Name"]] = by_disp[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        meta[did] = (r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    ids = sorted(meta)
    sgd = [i for i in ids if "sgd_momentum_kernel" in meta[i][0]]
    if len(sgd) >= 2:
        ids = [i for i in ids if sgd[-2] < i <= sgd[-1]]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(float)
    cnt = collections.Counter()
    for i in ids:
        name = meta[i][0].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:70]
        for k, v in by_disp[i].items():
            agg[name][k] += v
        dur[name] += meta[i][1] / 1e3
        cnt[name] += 1
    return agg, (dur, cnt)


def main():
    root = sys.argv[1]
    passes = sorted(glob.glob(os.path.join(root, "p[0-9]*")))
    allc = collections.defaultdict(dict)
    dur, cnt = {}, {}
    for d in passes:
        agg, dc = load_pass(d)
        if not agg:
            continue
        if not dur:
            dur, cnt = dc
        for k, v in agg.items():
            allc[k].update(v)
    tot = sum(dur.values())
    print(f"# one optimizer step, {sum(cnt.values())} dispatches, {tot / 1e3:.2f} ms kernel time (profiled: serialized)")
    print(f"{'kernel':70s} {'n':>4s} {'ms':>7s} {'%':>5s} {'mfma%':>6s} {'valu/mf':>7s} {'wait':>5s} {'instw':>5s} "
          f"{'lds_cf':>6s} {'rdGB':>7s} {'wrGB':>7s} {'TB/s':>6s} {'l2hit':>6s}")
    for k, t in sorted(dur.items(), key=lambda kv: -kv[1]):
        v = allc.get(k, {})
        g = lambda n: v.get(n, float("nan"))
        wc = g("SQ_WAVE_CYCLES")
        rd = 2 * g("FETCH_SIZE") / 1e9 * 1e3     # FETCH_SIZE is in KB
        wr = g("WRITE_SIZE") / 1e9 * 1e3
        tbs = (rd + wr) / (t / 1e6) / 1e3 if t > 0 else float("nan")
        print(f"{k:70s} {cnt[k]:4d} {t / 1e3:7.3f} {100 * t / tot:5.1f} "
              f"{100 * g('SQ_VALU_MFMA_BUSY_CYCLES') / max(g('GRBM_GUI_ACTIVE') * 4 * 32, 1):6.1f} "
              f"{g('SQ_INSTS_VALU') / max(g('SQ_INSTS_MFMA'), 1):7.2f} {g('SQ_WAIT_ANY') / wc:5.2f} "
              f"{g('SQ_WAIT_INST_ANY') / wc:5.2f} {g('SQ_LDS_BANK_CONFLICT') / max(g('SQ_LDS_IDX_ACTIVE'), 1):6.3f} "
              f"{rd:7.3f} {wr:7.3f} {tbs:6.2f} "
              f"{100 * g('TCC_HIT_sum') / max(g('TCC_HIT_sum') + g('TCC_MISS_sum'), 1):6.1f}")


if __name__ == "__main__":
    main()
