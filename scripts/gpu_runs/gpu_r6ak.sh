# round 6, call AK (final sources): rocprofv3 kernel trace + stats and HBM FETCH_SIZE / WRITE_SIZE passes of the
# regression bench lines (config 3, config 5, linear d = 1024), for the bench lines' roofline durations and traffic
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
bash scripts/gpu_prof.sh r6ak_logistic128 --config logistic128 --no-ess &&
bash scripts/gpu_prof.sh r6ak_linear512 --config linear512 --no-ess &&
bash scripts/gpu_prof.sh r6ak_linear1024 --config linear1024 --no-ess &&
echo all-done
