export OUT=r6_halo
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6_halo
timeout -k 10 300 python -u -m pytest tests/test_conv_halo_gpu.py tests/test_fullshape_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_halo/tests3.log 2>&1; tail -2 gpurun_out/r6_halo/tests3.log; PVA_TUNE_LOG=1 timeout -k 10 400 python bench.py > gpurun_out/r6_halo/bench.json 2> gpurun_out/r6_halo/bench.err; cat gpurun_out/r6_halo/bench.json; grep -c "halo224/d" gpurun_out/r6_halo/bench.err
