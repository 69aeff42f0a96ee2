#!/bin/bash
# non-temporal stores in bn_bwd_apply: probe A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2nt
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/pw_probe.py > gpurun_out/r2nt/p0.txt 2>&1 || { tail -20 gpurun_out/r2nt/p0.txt; exit 1; }
PVA_ELT_NT=1 timeout -k 10 200 python -u scripts/pw_probe.py > gpurun_out/r2nt/p1.txt 2>&1 || { tail -20 gpurun_out/r2nt/p1.txt; exit 1; }
paste gpurun_out/r2nt/p0.txt gpurun_out/r2nt/p1.txt | grep -E "bn_bwd|copy|fres"
