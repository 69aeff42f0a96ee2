#!/bin/bash
# PMC counters for the conv kernels of one microbenchmark layer (two counter passes, own runs).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ONLY=${ONLY:-res4.conv_a0}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
timeout -k 10 300 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d gpurun_out/pmc1 -o p1 -- python3 scripts/conv_bench.py --only $ONLY --iters 3 > gpurun_out/pmc1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc $P2 --kernel-trace --output-format csv -d gpurun_out/pmc2 -o p2 -- python3 scripts/conv_bench.py --only $ONLY --iters 3 > gpurun_out/pmc2.log 2>&1 || exit 1
ls gpurun_out/pmc1 gpurun_out/pmc2
