"""Summarise gpu_pmc.sh output: per conv kernel (last dispatch of each name) derived ratios."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
layers = sorted(set(os.path.basename(d).rsplit("_", 1)[0][4:] for d in glob.glob(os.path.join(root, "pmc_*_[0-9]"))))
for L in layers:
    vals = collections.defaultdict(dict)   # kernel -> counter -> value (last dispatch)
    dur = {}
    for i in range(1, 5):
        f = glob.glob(os.path.join(root, f"pmc_{L}_{i}", "*counter_collection.csv"))
        if not f:
            continue
        last = {}
        for r in csv.DictReader(open(f[0])):
            n = r["Kernel_Name"]
            if "conv_" not in n:
                continue
            key = n.replace("void (anonymous namespace)::", "").split("(")[0]
            did = int(r["Dispatch_Id"])
            if key not in last or did >= last[key][0]:
                if key in last and did > last[key][0]:
                    vals[key] = {k: v for k, v in vals[key].items() if not k.startswith(f"p{i}:")}
                last[key] = (did,)
                vals[key][f"p{i}:" + r["Counter_Name"]] = vals[key].get(f"p{i}:" + r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f"== {L}")
    for k, v in vals.items():
        g = lambda n: next((x for kk, x in v.items() if kk.split(":")[1] == n), float("nan"))
        wc = g("SQ_WAVE_CYCLES")
        print(f"  {k[:60]:60s} {dur.get(k, 0):7.1f}us  VALU/MFMA {g('SQ_INSTS_VALU') / max(g('SQ_INSTS_MFMA'), 1):5.2f}  "
              f"wait {g('SQ_WAIT_ANY') / wc:4.2f} instwait {g('SQ_WAIT_INST_ANY') / wc:4.2f}  "
              f"mfma_busy/gui {g('SQ_VALU_MFMA_BUSY_CYCLES') / max(g('GRBM_GUI_ACTIVE'), 1):5.2f}  "
              f"ldsconf {g('SQ_LDS_BANK_CONFLICT') / max(g('SQ_LDS_IDX_ACTIVE'), 1):4.2f}  "
              f"fetchGB {2 * g('FETCH_SIZE') / 1e6:6.3f} writeGB {g('WRITE_SIZE') / 1e6:6.3f} "
              f"L2hit {g('TCC_HIT_sum'):.3g}")
