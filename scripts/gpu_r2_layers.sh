#!/bin/bash
# per-op breakdown of the bench step (B=160) with and without conv_c BN folding
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2l
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/layer_profile.py --batch 160 --steps 2 > gpurun_out/r2l/fold.txt 2> gpurun_out/r2l/fold.err || { tail -20 gpurun_out/r2l/fold.err; exit 1; }
PVA_BN_FOLD_MIN_C=100000 timeout -k 10 300 python -u scripts/layer_profile.py --batch 160 --steps 2 > gpurun_out/r2l/nofold.txt 2> gpurun_out/r2l/nofold.err || { tail -20 gpurun_out/r2l/nofold.err; exit 1; }
head -1 gpurun_out/r2l/fold.txt gpurun_out/r2l/nofold.txt
