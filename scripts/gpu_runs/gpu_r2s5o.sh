# round 2 session 5: re-profile after the RAM changes moved the step-kernel source hash (metric kernel code
# unchanged): metric trace/traffic + VALU PMC on the driver's command, config-2 and config-4 VALU PMC, RAM d=32
# trace/traffic.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
G="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE"
bash scripts/gpu_prof.sh r2s5o_metric20 --gpus 1 --steps 20 --warmup 5 --no-ess || exit $?
PMC_GROUPS="$G" bash scripts/gpu_pmc.sh r2s5o_metric20 --gpus 1 --steps 20 --warmup 5 --no-ess || exit $?
PMC_GROUPS="$G" bash scripts/gpu_pmc.sh r2s5o_d3 --config d3 --steps 200 --warmup 20 --no-ess || exit $?
PMC_GROUPS="$G" bash scripts/gpu_pmc.sh r2s5o_hmc --config hmc1024 --steps 100 --warmup 10 --no-ess || exit $?
bash scripts/gpu_prof.sh r2s5o_ram32 --config ram32 --no-ess || exit $?
echo all-done
