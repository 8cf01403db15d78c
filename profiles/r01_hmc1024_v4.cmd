bash scripts/gpu_prof.sh r01_hmc1024_v4 --config hmc1024
# = rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r01_hmc1024_v4/trace -o run -- python3 bench.py --no-cpu-baseline --config hmc1024
#   rocprofv3 --pmc FETCH_SIZE ... and rocprofv3 --pmc WRITE_SIZE ... (separate passes, same command)
