bash scripts/gpu_prof.sh r01_metric_v3 --steps 1000 --warmup 100   (rocprofv3 --kernel-trace --stats; --pmc FETCH_SIZE; --pmc WRITE_SIZE; each -- python3 bench.py --no-cpu-baseline ...)
