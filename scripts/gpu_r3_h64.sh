#!/bin/bash
# persistent 64-channel halo conv: kernel tests vs fp32 PyTorch, then the conv_b micro-benchmark
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r3h64
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_halo_gpu.py > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python -u scripts/halo_bench.py --only 64 2>&1 | grep -v amdgpu.ids | tee $out/halo_bench.txt
