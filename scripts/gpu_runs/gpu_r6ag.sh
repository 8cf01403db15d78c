# round 6, call AG (final sources: tile skip + pairing): fp64 PMC of configs 3, 5 and linear d = 1024, VALU PMC of the small
# regression lines (the regression source hash covers csrc/*.hpp, ram_wave.hpp included)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6ag
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
export PMC_GROUPS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
run pmc_binomial 300 bash scripts/gpu_pmc.sh r6ag_binomial --config binomial --no-ess
run pmc_ramlinear 300 bash scripts/gpu_pmc.sh r6ag_ramlinear --config ramlinear --no-ess
export PMC_GROUPS="SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE;SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_LDS;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_LDS"
run pmc_log128 400 bash scripts/gpu_pmc.sh r6ag_log128 --config logistic128 --steps 20 --warmup 2 --no-ess
run pmc_lin512 600 bash scripts/gpu_pmc.sh r6ag_lin512 --config linear512 --steps 4 --warmup 100 --no-ess
run pmc_lin1024 600 bash scripts/gpu_pmc.sh r6ag_lin1024 --config linear1024 --no-ess
echo all-done
