#!/bin/bash
# PMC counters for the conv kernels of microbenchmark layers (own runs per counter pass; no trace domains).
#   ONLY="s.res4.conv_a0 s.res2.conv_c" BATCH=8 bash scripts/gpu_pmc.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
P3="FETCH_SIZE"
P4="WRITE_SIZE TCC_HIT_sum"
for L in ${ONLY:-s.res4.conv_a0}; do
  i=0
  for P in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pmc_${L}_$i -o p -- python3 scripts/conv_bench.py --only $L --iters 2 --batch ${BATCH:-8} > gpurun_out/pmc_${L}_$i.log 2>&1 || { tail -5 gpurun_out/pmc_${L}_$i.log; exit 1; }
  done
done
ls gpurun_out | grep pmc_ | head -40
