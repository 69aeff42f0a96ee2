#!/bin/bash
# Fresh PMC pass over one steady-state step at B=64 (current kernels), summary only (raw CSVs removed).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PMC_OUT=r2f/pmc BATCH=64
bash scripts/gpu_pmc_step.sh > gpurun_out/r2f_pmc_head.txt 2>&1 || { tail -20 gpurun_out/r2f_pmc_head.txt; exit 1; }
rm -rf gpurun_out/r2f/pmc/p1 gpurun_out/r2f/pmc/p2 gpurun_out/r2f/pmc/p3 gpurun_out/r2f/pmc/p4
head -30 gpurun_out/r2f/pmc/summary.txt
