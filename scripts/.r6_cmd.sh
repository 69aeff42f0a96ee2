export OUT=r6_gen2
bash scripts/gpu_run.sh layers bench
