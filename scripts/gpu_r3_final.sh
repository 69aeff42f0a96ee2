#!/bin/bash
# round-3 final validation: smoke, every GPU test, headline bench (synthetic and host-fed), the reference CLI
# (run.py) at the headline shape on a synthetic corpus, steady-state kernel trace, per-op profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r3final
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
PVA_TUNE_LOG=1 timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 400 python bench.py --source host > $out/bench_host.json 2> $out/bench_host.err || { tail -30 $out/bench_host.err; exit 1; }
cat $out/bench_host.json
timeout -k 10 600 python -u run.py --synthetic --is_slowfast --num_frames 32 --sampling_rate 2 --crop_size 224 \
  --batch_size 160 --gradient_accumulation_steps 1 --mixed_precision bf16 --num_epochs 2 --limit_train_batches 8 \
  --limit_val_batches 0 --num_workers 8 --synthetic_videos 1280 --output_dir /tmp/pva_run > $out/run_py.log 2>&1 || { tail -30 $out/run_py.log; exit 1; }
grep -i "clips/s\|epoch" $out/run_py.log | tail -4
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $out/prof -o step -- python3 bench.py --steps 3 --warmup 3 > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
f=$(ls $out/prof/*/step_kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] || f=$(ls $out/prof/step_kernel_trace.csv)
python scripts/steady_state_kernels.py "$f" --steps 2 > $out/kernels_steady_state.txt && head -3 $out/kernels_steady_state.txt
rm -f "$f"
timeout -k 10 300 python -u scripts/layer_profile.py --batch 160 --steps 2 > $out/layers_b160.txt 2> $out/layers.err || { tail -20 $out/layers.err; exit 1; }
head -1 $out/layers_b160.txt
