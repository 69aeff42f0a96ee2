export OUT=r6_epi2
bash scripts/gpu_run.sh smoke tests bench
