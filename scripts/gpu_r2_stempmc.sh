#!/bin/bash
# LDS bank-conflict / MFMA-busy counters of the stem weight-gradient kernels only (one rocprofv3 pass)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r2sp
mkdir -p $out
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES --kernel-include-regex "stem_wgrad" --kernel-trace --output-format csv -d $out/p -o p -- python3 bench.py --steps 2 --warmup 1 --batch 32 > $out/p.log 2>&1 || { tail -5 $out/p.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/r2sp/p/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    agg[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k, "lds_conflict/active = %.3f" % (v["SQ_LDS_BANK_CONFLICT"] / max(1, v["SQ_LDS_IDX_ACTIVE"])),
          "wait = %.2f" % (v["SQ_WAIT_ANY"] / max(1, v["SQ_WAVE_CYCLES"])))
PY
rm -rf $out/p
