bash scripts/gpu_prof.sh r01_d3_v2 --config d3   (rocprofv3 --kernel-trace --stats; --pmc FETCH_SIZE; --pmc WRITE_SIZE; each -- python3 bench.py --no-cpu-baseline --config d3)
