#!/bin/bash
# Stock PyTorch baseline on one MI355X + a rocprofv3 kernel summary.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python scripts/baseline_torch.py --batch 8 --steps 10 --warmup 3 > gpurun_out/base_b8.json 2> gpurun_out/base_b8.err || exit $?
timeout -k 10 400 python scripts/baseline_torch.py --batch 8 --steps 10 --warmup 3 --channels-last > gpurun_out/base_b8_cl.json 2> gpurun_out/base_b8_cl.err || exit $?
timeout -k 10 500 python scripts/baseline_torch.py --batch 32 --steps 6 --warmup 2 > gpurun_out/base_b32.json 2> gpurun_out/base_b32.err || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_base -o base --output-format csv -- python3 scripts/baseline_torch.py --batch 8 --steps 3 --warmup 2 > gpurun_out/prof_base.log 2>&1 || exit $?
cat gpurun_out/base_*.json
