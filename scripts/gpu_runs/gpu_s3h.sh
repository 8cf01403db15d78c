# rocprofv3 of config 3 on the current build (no elementwise fences) + the default bench line.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_prof.sh r01_logistic128_v4 --config logistic128 || exit 1
timeout -k 10 400 python3 bench.py > gpurun_out/s3h_bench.log 2>&1 || { echo "bench failed"; exit 1; }
echo all-done
