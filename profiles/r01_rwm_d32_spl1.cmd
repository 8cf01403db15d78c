rocprofv3 --kernel-trace --stats --output-format csv -- python3 bench.py --no-cpu-baseline --steps 200 --warmup 0 --spl 1   (then --pmc FETCH_SIZE, --pmc WRITE_SIZE passes)
