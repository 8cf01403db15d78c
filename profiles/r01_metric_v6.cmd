bash scripts/gpu_prof.sh r01_metric_v6
# = rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r01_metric_v6/trace -o run -- python3 bench.py --no-cpu-baseline
#   rocprofv3 --pmc FETCH_SIZE ... and rocprofv3 --pmc WRITE_SIZE ... (separate passes, same command)
