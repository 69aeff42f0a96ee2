#!/bin/bash
# after a kernel change: GPU tests (all, or the files in $TESTS), headline bench with the tuner log, per-op profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${OUT:-r3step}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
PVA_TUNE_LOG=1 timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
cat $out/bench.json
grep -c "halo224/p" $out/bench.err || true
timeout -k 10 300 python -u scripts/layer_profile.py --batch 160 --steps 2 > $out/layers_b160.txt 2> $out/layers.err || { tail -20 $out/layers.err; exit 1; }
head -2 $out/layers_b160.txt
