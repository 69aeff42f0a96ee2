export OUT=r6_gen3
bash scripts/gpu_run.sh pmc fp16 host
