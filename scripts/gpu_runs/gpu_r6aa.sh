# round 6, call AA: VALU PMC of the small regression lines (binomial: glm_rwm<1, 1>; ramlinear: glm_ram<1, 1>), then
# their bench lines against the profiles (bench.py names the larger of the VALU and MFMA fractions)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6aa
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
export PMC_GROUPS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
run pmc_binomial 300 bash scripts/gpu_pmc.sh r6aa_binomial --config binomial --no-ess
run pmc_ramlinear 300 bash scripts/gpu_pmc.sh r6aa_ramlinear --config ramlinear --no-ess
echo all-done
