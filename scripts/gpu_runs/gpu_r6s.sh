# round 6, call S (final build; rerun as call V after the last regression-kernel change): fp64-datapath PMC of the regression configs 3 and 5 and linear d = 1024
# (bench.py's fp64_combined: profiles/fp64.json, scripts/summarize_fp64.py)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${CALL:-r6s}
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
G="SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE;SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_LDS;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_LDS"
export PMC_GROUPS="$G"
run pmc_log128 400 bash scripts/gpu_pmc.sh ${CALL:-r6s}_log128 --config logistic128 --steps 20 --warmup 2 --no-ess
run pmc_lin512 600 bash scripts/gpu_pmc.sh ${CALL:-r6s}_lin512 --config linear512 --steps 4 --warmup 100 --no-ess
run pmc_lin1024 600 bash scripts/gpu_pmc.sh ${CALL:-r6s}_lin1024 --config linear1024 --no-ess
echo all-done
