cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 1000 bash scripts/gpu_pmc.sh r01_logistic128 --config logistic128 --steps 10 --warmup 1
