#!/bin/bash
# the reference CLI (run.py) at the headline shape (SlowFast-R50 32x2x224, B=160, bf16) on a raw-frame .npy corpus:
# native C++ reader (num_workers 0) -> pinned memory -> H2D copy stream -> on-device preprocessing -> fused step.
# The corpus is bench.py's 96 random videos, linked 20x into a 1920-video train split (val: the same list).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r3runpy
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --source host --steps 2 --warmup 1 > $out/bench_host.json 2> $out/bench_host.err || { tail -20 $out/bench_host.err; exit 1; }
src=/tmp/pva_bench_corpus/64x256x340_96/train
dst=/tmp/pva_runpy_corpus
rm -rf $dst && mkdir -p $dst/train
for c in $(ls $src); do
  mkdir -p $dst/train/$c
  for f in $src/$c/*.npy; do b=$(basename $f .npy); for r in $(seq 0 19); do ln -s $f $dst/train/$c/${b}_$r.npy; done; done
done
ln -s $dst/train $dst/val
timeout -k 10 600 python -u run.py --data_dir $dst --is_slowfast --num_frames 32 --sampling_rate 2 --crop_size 224 \
  --batch_size 160 --gradient_accumulation_steps 1 --mixed_precision bf16 --num_epochs 3 --limit_train_batches 10 \
  --limit_val_batches 0 --num_workers 0 --output_dir /tmp/pva_run --quiet > $out/run_py.log 2>&1 || { tail -30 $out/run_py.log; exit 1; }
grep -i "clips/s" $out/run_py.log | tail -4
