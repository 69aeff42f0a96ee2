#!/bin/bash
# PMC passes over one steady-state bench step at the headline batch (one run per pass, no trace domains), plus the
# SQ pass over the conv_b micro-benchmark (64/128-channel halo-staged kernels and their alternatives)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r3pmc; mkdir -p $o
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
for i in ${PASSES:-2 3}; do
  case $i in 1) P="$P1";; 2) P="FETCH_SIZE";; 3) P="WRITE_SIZE";; 4) P="TCC_HIT_sum TCC_MISS_sum";; esac
  timeout -k 10 600 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $o/p$i -o p -- python3 bench.py --steps 2 --warmup 1 > $o/p$i.log 2>&1 || { tail -5 $o/p$i.log; exit 1; }
  echo pass $i done
done
if [ -n "$HALO" ]; then
  timeout -k 10 600 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $o/halo -o h -- python3 scripts/halo_bench.py --only 64,128 > $o/halo.log 2>&1 || { tail -5 $o/halo.log; exit 1; }
  grep -v amdgpu.ids $o/halo.log | tail -20
fi
