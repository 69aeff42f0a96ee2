export OUT=r6_pwp
bash scripts/gpu_run.sh smoke tests bench
