bash scripts/gpu_prof.sh r01_hmc1024_v2 --config hmc1024   (rocprofv3 --kernel-trace --stats; --pmc FETCH_SIZE; --pmc WRITE_SIZE; each -- python3 bench.py --no-cpu-baseline --config hmc1024)
