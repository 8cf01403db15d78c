rocprofv3 --kernel-trace --stats --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1000 --warmup 0   (then --pmc FETCH_SIZE, --pmc WRITE_SIZE passes)
