bash scripts/gpu_prof.sh r01_linear512_v2 --config linear512   (rocprofv3 --kernel-trace --stats; --pmc FETCH_SIZE; --pmc WRITE_SIZE; each -- python3 bench.py --no-cpu-baseline --config linear512)
