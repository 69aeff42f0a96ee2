"""Per-kernel-name summary of rocprofv3 --pmc passes over scripts/pw_pmc_probe.py (mean per dispatch,
first dispatch of each kernel skipped as warm-up).

    python scripts/pmc_probe_summary.py gpurun_out/r2pwpmc
Derived: DRAM read / write GB (32-B sectors), achieved TB/s, mean TCP->TCC read latency (cycles),
mean L2->EA read requests in flight."""
import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for d in sorted(glob.glob(os.path.join(root, "p[0-9]*"))):
        f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not f:
            continue
        rows = list(csv.DictReader(open(f[0])))
        disp = collections.defaultdict(dict)
        meta = {}
        for r in rows:
            i = int(r["Dispatch_Id"])
            disp[i][r["Counter_Name"]] = disp[i].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            kn = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            meta[i] = (kn[:60], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        seen = collections.Counter()
        for i in sorted(meta):
            name = meta[i][0]
            seen[name] += 1
            if seen[name] == 1:
                continue
            for k, v in disp[i].items():
                per[name][k].append(v)
            dur[name].append(meta[i][1])
    for name, cs in per.items():
        avg = {k: sum(v) / len(v) for k, v in cs.items()}
        t = sum(dur[name]) / len(dur[name]) * 1e-9
        out = ["%-60s %8.1f us" % (name, t * 1e6)]
        rd = avg.get("TCC_EA0_RDREQ_DRAM_32B_sum")
        wr = avg.get("TCC_EA0_WRREQ_WRITE_DRAM_32B_sum")
        if rd is not None and wr is not None:
            out.append("dram rd %.2f GB wr %.2f GB  %.2f TB/s" % (rd * 32e-9, wr * 32e-9, (rd + wr) * 32 / t * 1e-12))
        if avg.get("TCP_TCC_READ_REQ_sum"):
            out.append("rd lat %.0f cyc" % (avg["TCP_TCC_READ_REQ_LATENCY_sum"] / avg["TCP_TCC_READ_REQ_sum"]))
        if avg.get("TCP_TCC_WRITE_REQ_sum"):
            out.append("wr lat %.0f cyc" % (avg["TCP_TCC_WRITE_REQ_LATENCY_sum"] / avg["TCP_TCC_WRITE_REQ_sum"]))
        if avg.get("TCC_EA0_RDREQ_LEVEL_sum") and avg.get("GRBM_GUI_ACTIVE"):
            out.append("ea rd in flight %.0f" % (avg["TCC_EA0_RDREQ_LEVEL_sum"] / avg["GRBM_GUI_ACTIVE"]))
        if avg.get("TCC_HIT_sum") is not None and avg.get("TCC_MISS_sum"):
            out.append("l2hit %.2f" % (avg["TCC_HIT_sum"] / (avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])))
        if avg.get("SQ_WAVE_CYCLES"):
            wc = avg["SQ_WAVE_CYCLES"]
            out.append("wait %.2f issue-wait %.2f valu %.2f vmem %.2f (of wave-cycles)" % (
                avg.get("SQ_WAIT_ANY", 0) / wc, avg.get("SQ_WAIT_INST_ANY", 0) / wc,
                avg.get("SQ_ACTIVE_INST_VALU", 0) / wc, avg.get("SQ_ACTIVE_INST_VMEM", 0) / wc))
        print("  ".join(out))
        print("    " + " ".join("%s=%.3g" % kv for kv in sorted(avg.items())))


if __name__ == "__main__":
    main()
