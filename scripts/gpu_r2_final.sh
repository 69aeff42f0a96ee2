#!/bin/bash
# end-of-session validation: smoke(), full GPU suite, headline bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r2fin
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/gt.log 2>&1 || { tail -40 $out/gt.log; exit 1; }
tail -1 $out/gt.log
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
cat $out/bench.json
