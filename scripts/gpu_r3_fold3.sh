#!/bin/bash
# single-launch BN-fold kernels (3+4 -> 1+2 launches per folded layer) + 1024-thread finalize: GPU tests, bench, kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r3fold3
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_bnfold_gpu.py tests/test_bn_pool_kernels_gpu.py tests/test_fused_gpu.py tests/test_blocks_gpu.py tests/test_fullshape_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 300 python bench.py > $out/bench2.json 2> $out/bench2.err || { tail -30 $out/bench2.err; exit 1; }
cat $out/bench2.json
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $out/prof -o step -- python3 bench.py --steps 3 --warmup 3 > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
f=$(ls $out/prof/*/step_kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] || f=$(ls $out/prof/step_kernel_trace.csv)
python scripts/steady_state_kernels.py "$f" --steps 2 > $out/kernels_steady_state.txt && head -3 $out/kernels_steady_state.txt
grep "finalize2\|bnfold" $out/kernels_steady_state.txt | head -4
mv "$f" $out/step_kernel_trace.csv
PVA_BNFOLD_FUSED=0 timeout -k 10 300 python bench.py > $out/bench_nofold3.json 2> $out/bench_nofold3.err || { tail -30 $out/bench_nofold3.err; exit 1; }
cat $out/bench_nofold3.json
