# round 4 profiles for the final step-kernel sources: VALU PMC passes of the driver's metric command (20 steps) and
# of 1 000 steps, the kernel trace + FETCH_SIZE / WRITE_SIZE passes of the driver's command, VALU of d3 and hmc1024
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4j
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run pmc_m20 400 bash scripts/gpu_pmc.sh r4j_metric20 --no-ess
run prof_m20 400 bash scripts/gpu_prof.sh r4j_metric20 --no-ess
run pmc_m1000 400 bash scripts/gpu_pmc.sh r4j_metric1000 --steps 1000 --no-ess
run pmc_d3 400 bash scripts/gpu_pmc.sh r4j_d3 --config d3 --no-ess
run pmc_hmc1024 500 bash scripts/gpu_pmc.sh r4j_hmc1024 --config hmc1024 --no-ess
echo all-done
G="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE;SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_WAVES;FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_WRITE_REQ_sum;TA_BUSY_avr TA_TA_BUSY_sum"
PMC_GROUPS="$G" run pmc_ram256 600 bash scripts/gpu_pmc.sh r4j_ram256 --config ram256 --steps 20 --no-ess
echo all-done-2
