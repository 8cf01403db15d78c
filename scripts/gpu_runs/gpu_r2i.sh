# round 2: PMC of the config-1 kernel (one block: wave 0 consumes, waves 1-3 generate)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
PMC_GROUPS="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE;SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INSTS_BRANCH" \
  bash scripts/gpu_pmc.sh r2_readme --config readme --thinning 100 --no-ess || exit $?
echo all-done
