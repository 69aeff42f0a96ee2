export OUT=r6_f32d
export KSTATS_ARGS="--precision fp32 --batch 64"
PVA_ARMS=f32_direct_k=0 bash scripts/gpu_run.sh kstats && mv gpurun_out/r6_f32d/kernel_stats.csv gpurun_out/r6_f32d/kernel_stats_mfma.csv && bash scripts/gpu_run.sh kstats
