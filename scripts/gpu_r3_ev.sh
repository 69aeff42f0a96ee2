#!/bin/bash
# evidence runs: (1) host-fed bench under a kernel + memory-copy trace (H2D copies vs compute), (2) two gloo ranks
# sharing the GPU under a marker trace (per-stage and per-bucket all-reduce ROCTx ranges)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r3ev
mkdir -p $out
timeout -k 10 500 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $out/h2d -o h -- python3 bench.py --source host --steps 4 --warmup 3 > $out/h2d.log 2>&1 || { tail -20 $out/h2d.log; exit 1; }
grep '"metric"' $out/h2d.log | tail -1
PVA_DIST_BACKEND=gloo timeout -k 10 500 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $out/dp2 -o d -- python3 bench.py --gpus 2 --batch 32 --steps 3 --warmup 2 > $out/dp2.log 2>&1 || { tail -20 $out/dp2.log; exit 1; }
grep '"metric"' $out/dp2.log | tail -1
ls -R $out | head -30
