set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "stem" > gpurun_out/t_stem.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 12 --warmup 2 > gpurun_out/bench_n.json 2> gpurun_out/bench_n.err &&
timeout -k 10 300 python scripts/layer_profile.py --batch 96 > gpurun_out/layers96n.txt 2>&1
rc=$?; tail -3 gpurun_out/t_stem.log; cat gpurun_out/bench_n.json; grep -E "^b0\.p1" gpurun_out/layers96n.txt; exit $rc
