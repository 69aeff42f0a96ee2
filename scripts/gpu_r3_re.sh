#!/bin/bash
# round-3 re-entry: smoke, all GPU tests, headline bench, host-fed bench, kernel + marker trace of a short run
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r3re
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 400 python bench.py --source host > $out/bench_host.json 2> $out/bench_host.err || { tail -30 $out/bench_host.err; exit 1; }
cat $out/bench_host.json
timeout -k 10 500 rocprofv3 --kernel-trace --marker-trace --stats -d $out/prof -o step --output-format csv -- python3 bench.py --steps 3 --warmup 3 > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
f=$(ls $out/prof/*/step_kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] || f=$(ls $out/prof/step_kernel_trace.csv)
python scripts/steady_state_kernels.py "$f" --steps 2 > $out/kernels_steady_state.txt && head -5 $out/kernels_steady_state.txt
ls -R $out/prof | head -20
