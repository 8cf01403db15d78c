# rocprofv3 kernel-trace/stats + FETCH_SIZE/WRITE_SIZE passes of config 3 (logistic MALA) and the config-4 shard
# at the bench defaults; a quick parity check of the regression kernels first.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -k "glm or golden" --timeout 120 --timeout-method thread > gpurun_out/s3d_tests.log 2>&1 || { echo "tests failed"; exit 1; }
bash scripts/gpu_prof.sh r01_logistic128_v3 --config logistic128 || exit 1
bash scripts/gpu_prof.sh r01_hmc1024_v3 --config hmc1024 || exit 1
echo all-done
