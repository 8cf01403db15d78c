# round 3: fp64 datapath PMC of the regression kernels (config 3 logistic MALA, config 5 linear HMCDA adapted)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3k
mkdir -p $O
G="SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE;SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_LDS;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_SALU"
PMC_GROUPS="$G" timeout -k 10 900 bash scripts/gpu_pmc.sh r3k_log128 --config logistic128 --steps 20 --warmup 2 --no-ess > $O/pmc_log128.log 2>&1 || exit 1
PMC_GROUPS="$G" timeout -k 10 900 bash scripts/gpu_pmc.sh r3k_lin512 --config linear512 --steps 10 --no-ess > $O/pmc_lin512.log 2>&1 || exit 1
echo all-done
