# round 6, call A: GPU suite + smoke, then VALU PMC passes of the separable-target bench lines (bench.py's VALU
# roofline: profiles/valu.json) and the kernel trace + HBM traffic of the driver's 20-step command
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6a
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run gputests 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run pmc_metric20 300 bash scripts/gpu_pmc.sh r6a_metric20 --steps 20 --warmup 5 --no-ess
run prof_metric20 400 bash scripts/gpu_prof.sh r6a_metric20 --steps 20 --warmup 5 --no-ess
export PMC_GROUPS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
run pmc_metric1000 300 bash scripts/gpu_pmc.sh r6a_metric1000 --steps 1000 --no-ess
run pmc_d3 300 bash scripts/gpu_pmc.sh r6a_d3 --config d3 --no-ess
run pmc_hmc1024 300 bash scripts/gpu_pmc.sh r6a_hmc1024 --config hmc1024 --no-ess
echo all-done
