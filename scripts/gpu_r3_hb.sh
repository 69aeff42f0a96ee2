#!/bin/bash
# halo conv micro-benchmark at the B=160 conv_b shapes (+ kernel tests)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r3hb
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_halo_gpu.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 400 python -u scripts/halo_bench.py "$@" 2>&1 | grep -v amdgpu.ids | tee $out/halo_bench.txt
# PMC (SQ counters, one pass, no trace domains) of the C=64 / C=128 conv_b kernels at B=64
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 240 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $out/pmc/p1 -o p -- python3 scripts/halo_bench.py --only 64,128 --batch 64 > $out/pmc_p1.log 2>&1 || { tail -5 $out/pmc_p1.log; exit 1; }
python3 scripts/pmc_step_summary.py $out/pmc > $out/pmc_summary.txt && head -30 $out/pmc_summary.txt
