#!/bin/bash
# PMC counters over one steady-state bench.py step (4 passes, each its own run; no trace domains).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${PMC_OUT:-pmc_step}
mkdir -p $OUT
B=${BATCH:-32}
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P2="FETCH_SIZE"
P3="WRITE_SIZE"
P4="TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -k 10 420 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/p$i -o p -- python3 bench.py --steps 2 --warmup 1 --batch $B > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
done
python3 scripts/pmc_step_summary.py $OUT > $OUT/summary.txt && head -45 $OUT/summary.txt
