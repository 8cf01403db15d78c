# round 2 session 4: metric kernel VALU PMC + traffic on the driver's command after the block-per-chain change
# (the step-kernel source hash moved; the metric kernel's code is unchanged).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
bash scripts/gpu_prof.sh r2s4y_metric20 --gpus 1 --steps 20 --warmup 5 --no-ess || exit $?
PMC_GROUPS="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE;SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32;SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  bash scripts/gpu_pmc.sh r2s4y_metric20 --gpus 1 --steps 20 --warmup 5 --no-ess || exit $?
echo all-done
