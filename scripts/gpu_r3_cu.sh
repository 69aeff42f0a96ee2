#!/bin/bash
# stream-placement A/B at the headline config: default two-stream schedule vs the fast pathway confined to a CU
# subset (hipExtStreamCreateWithCUMask), with / without the slow pathway on the complementary CUs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r3cu
mkdir -p $out
export TMPDIR=/tmp
run() {   # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $out/$name.json 2> $out/$name.err || { tail -20 $out/$name.err; exit 1; }
  echo "$name $(python -c "import json,sys; d=json.load(open('$out/$name.json')); print(d['value'], d['ms_per_step'])")"
}
run base PVA_NOOP=1
run side64 PVA_SIDE_CUS=64
run side64c PVA_SIDE_CUS=64 PVA_MAIN_CU_COMPLEMENT=1
run side128c PVA_SIDE_CUS=128 PVA_MAIN_CU_COMPLEMENT=1
run prio PVA_SIDE_PRIORITY=-1
# PMC pass 1 (SQ + GRBM) over one steady-state step at the headline batch
if [ -n "$PMC" ]; then
  o=gpurun_out/r3pmc; mkdir -p $o
  timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $o/p1 -o p -- python3 bench.py --steps 2 --warmup 1 > $o/p1.log 2>&1 || { tail -5 $o/p1.log; exit 1; }
  echo pmc1 done
fi
