#!/bin/bash
# PMC counters of the direct conv kernel on one layer (own rocprofv3 run per counter pass).
#   SHAPE=f.res2.conv_b CFG=direct2048 bash scripts/gpu_pmc_direct.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_VMEM_RD"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
P3="FETCH_SIZE"
P4="WRITE_SIZE TCC_HIT_sum"
S=${SHAPE:-f.res2.conv_b}
timeout -k 10 120 python3 scripts/direct_bench.py --shape $S --cfg ${CFG:-direct2048} > gpurun_out/pmcd_${S}_time.log 2>&1 || exit 1
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmcd_${S}_$i -o p -- python3 scripts/direct_bench.py --shape $S --cfg ${CFG:-direct2048} --iters 2 > gpurun_out/pmcd_${S}_$i.log 2>&1 || { tail -5 gpurun_out/pmcd_${S}_$i.log; exit 1; }
done
