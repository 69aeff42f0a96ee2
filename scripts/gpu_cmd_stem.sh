set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "stem" > gpurun_out/t_stem.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 12 --warmup 2 > gpurun_out/bench_o.json 2> gpurun_out/bench_o.err &&
timeout -k 10 300 python scripts/layer_profile.py --batch 96 > gpurun_out/layers96o.txt 2>&1
rc=$?; tail -3 gpurun_out/t_stem.log; cat gpurun_out/bench_o.json; grep -E "^b0\." gpurun_out/layers96o.txt; exit $rc
