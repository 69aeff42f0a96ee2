export OUT=r6_final2
bash scripts/gpu_run.sh smoke tests bench
