set -o pipefail
mkdir -p gpurun_out
for sh in s.res2.conv_c s.res3.conv_c; do for cfg in 280 25; do for ns in "" "--nostore" "--nostore --nostats"; do
timeout -k 10 60 python scripts/direct_bench.py --shape $sh --cfg $cfg --affine 1 $ns 2>&1 | grep -v amdgpu.ids || exit 1
done; done; done > gpurun_out/convc.txt
cat gpurun_out/convc.txt
