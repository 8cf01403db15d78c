bash scripts/gpu_prof.sh r01_logistic128_v4 --config logistic128
# = rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r01_logistic128_v4/trace -o run -- python3 bench.py --no-cpu-baseline --config logistic128
#   rocprofv3 --pmc FETCH_SIZE ... and rocprofv3 --pmc WRITE_SIZE ... (separate passes, same command)
