#!/bin/bash
# Autotuner candidate table for every conv geometry of one bench step (PVA_TUNE_LOG=1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/${OUT:-tunelog}
PVA_TUNE_LOG=1 timeout -k 10 400 python bench.py --steps 2 --warmup 1 --batch ${BATCH:-96} > gpurun_out/${OUT:-tunelog}/bench.json 2> gpurun_out/${OUT:-tunelog}/tune.log || { tail -20 gpurun_out/${OUT:-tunelog}/tune.log; exit 1; }
cat gpurun_out/${OUT:-tunelog}/bench.json; grep -c tune gpurun_out/${OUT:-tunelog}/tune.log
