# round 2 session 4: VALU PMC passes of the config-2 (d=3 RWM) and config-4 (d=1024 HMC) step kernels, so their bench
# lines carry the measured VALU roofline like the metric's.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
G="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE"
PMC_GROUPS="$G" bash scripts/gpu_pmc.sh r2s4z_d3 --config d3 --steps 200 --warmup 20 --no-ess || exit $?
PMC_GROUPS="$G" bash scripts/gpu_pmc.sh r2s4z_hmc --config hmc1024 --steps 100 --warmup 10 --no-ess || exit $?
timeout -k 10 200 python3 bench.py --config d3 --no-ess > gpurun_out/s4z_d3.log 2>&1 || exit 1
echo all-done
