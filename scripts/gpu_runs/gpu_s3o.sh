# rocprofv3 (kernel trace + FETCH_SIZE + WRITE_SIZE passes) of the metric workload and the config-4 shard on the final build.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_prof.sh r01_metric_v6 || exit 1

echo all-done
