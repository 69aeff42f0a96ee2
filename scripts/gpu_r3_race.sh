#!/bin/bash
# gradient reproducibility across stream schedules (small batch) + small-batch trajectory vs the oracles
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r3race
mkdir -p $out
export TMPDIR=/tmp
B=4 timeout -k 10 300 python -u scripts/diag_ms_race.py 2>&1 | grep -v amdgpu.ids | grep -v "^   " > $out/race_b4.log || exit 1
B=4 DET=1 timeout -k 10 300 python -u scripts/diag_ms_race.py 2>&1 | grep -v amdgpu.ids | grep -v "^   " > $out/race_b4_det.log || exit 1
B=32 timeout -k 10 300 python -u scripts/diag_ms_race.py 2>&1 | grep -v amdgpu.ids | grep -v "^   " > $out/race_b32.log || exit 1
cat $out/race_*.log
timeout -k 10 600 python -u scripts/diag_small_batch.py > $out/small_batch.log 2>&1 || { tail $out/small_batch.log; exit 1; }
tail -4 $out/small_batch.log
