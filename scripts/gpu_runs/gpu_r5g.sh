# round 5 final build, call A: GPU suite + smoke, VALU PMC passes of the lane/pair/wave-per-chain configs (bench.py's
# VALU roofline), kernel trace + HBM traffic of the driver's 20-step command
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5g
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run gputests 700 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run pmc_metric20 300 bash scripts/gpu_pmc.sh r5g_metric20 --steps 20 --warmup 5 --no-ess
run pmc_metric1000 300 bash scripts/gpu_pmc.sh r5g_metric1000 --steps 1000 --no-ess
run pmc_d3 300 bash scripts/gpu_pmc.sh r5g_d3 --config d3 --no-ess
run pmc_hmc1024 300 bash scripts/gpu_pmc.sh r5g_hmc1024 --config hmc1024 --no-ess
run pmc_bare_normal 300 bash scripts/gpu_pmc.sh r5g_bare_normal --config bare_normal --no-ess
run pmc_mala32 300 bash scripts/gpu_pmc.sh r5g_mala32 --sampler mala --no-ess
run pmc_hmc32 300 bash scripts/gpu_pmc.sh r5g_hmc32 --sampler hmc --no-ess
run prof_metric20 400 bash scripts/gpu_prof.sh r5g_metric20 --steps 20 --warmup 5 --no-ess
echo all-done
