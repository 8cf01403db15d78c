bash scripts/gpu_prof.sh r01_linear512 --config linear512 --steps 4 --warmup 1   (rocprofv3 --kernel-trace --stats; --pmc FETCH_SIZE; --pmc WRITE_SIZE; each -- python3 bench.py --no-cpu-baseline ...)
