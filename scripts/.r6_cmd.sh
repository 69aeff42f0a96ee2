export OUT=r6_nsc
bash scripts/gpu_run.sh smoke tests bench
