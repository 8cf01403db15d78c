# round 3, session 2: re-record the profiles bench.py prices its rooflines with, for the current step-kernel
# sources (VALU PMC: driver's 20-step command, 1000 steps, config 2, config 4; fp64 PMC: configs 3 and 5;
# trace + FETCH/WRITE of the driver's command)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3t
mkdir -p $O
timeout -k 10 600 bash scripts/gpu_prof.sh r3t_metric20 --steps 20 --warmup 5 --no-ess > $O/prof20.log 2>&1 || exit 1
timeout -k 10 600 bash scripts/gpu_pmc.sh r3t_metric20 --steps 20 --warmup 5 --no-ess > $O/pmc20.log 2>&1 || exit 1
timeout -k 10 600 bash scripts/gpu_pmc.sh r3t_metric1000 --no-ess > $O/pmc1000.log 2>&1 || exit 1
timeout -k 10 600 bash scripts/gpu_pmc.sh r3t_d3 --config d3 --no-ess > $O/pmcd3.log 2>&1 || exit 1
timeout -k 10 900 bash scripts/gpu_pmc.sh r3t_hmc1024 --config hmc1024 --no-ess > $O/pmch.log 2>&1 || exit 1
G="SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE;SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_LDS;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_SALU"
PMC_GROUPS="$G" timeout -k 10 900 bash scripts/gpu_pmc.sh r3t_log128 --config logistic128 --steps 20 --warmup 2 --no-ess > $O/pmc_log128.log 2>&1 || exit 1
PMC_GROUPS="$G" timeout -k 10 900 bash scripts/gpu_pmc.sh r3t_lin512 --config linear512 --steps 10 --no-ess > $O/pmc_lin512.log 2>&1 || exit 1
echo all-done
