#!/bin/bash
# current-kernel numbers for the other SURVEY model configs: SlowFast-R101 32x2x256 (B=48) and the 64-frame
# SlowFast-R50 64x2x224 (B=24, grad-accum 4) — round-1 numbers in profiles/r1_sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r2v
mkdir -p $out
timeout -k 10 420 python bench.py --depth 101 --crop 256 --batch 48 --steps 12 --warmup 2 > $out/r101_256_b48.json 2> $out/r101.err || { tail -10 $out/r101.err; exit 1; }
cut -c1-200 $out/r101_256_b48.json
timeout -k 10 420 python bench.py --frames 64 --batch 24 --grad-accum 4 --steps 12 --warmup 2 > $out/r50_64x2_gas4_b24.json 2> $out/r64.err || { tail -10 $out/r64.err; exit 1; }
cut -c1-200 $out/r50_64x2_gas4_b24.json
