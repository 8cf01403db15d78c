# PMC passes (VALU / MFMA issue, LDS, busy cycles) for the metric kernel, config 3 and config 4.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/gpu_pmc.sh metric --steps 200 --warmup 10 || exit $?
bash scripts/gpu_pmc.sh log128 --config logistic128 --steps 40 --warmup 2 || exit $?
bash scripts/gpu_pmc.sh h1024 --config hmc1024 --steps 200 --warmup 10 || exit $?
echo all-done
