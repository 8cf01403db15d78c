# round 6, call B: VALU PMC of the remaining separable lines, fp64-datapath PMC of the regression configs
# (bench.py's fp64_combined: profiles/fp64.json)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6b
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run gputests 600 python3 -u -m pytest tests/test_hook_protocol.py tests/test_task_streams.py tests/test_seqmc.py tests/test_sharded_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
export PMC_GROUPS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
run pmc_bare_normal 300 bash scripts/gpu_pmc.sh r6b_bare_normal --config bare_normal --no-ess
run pmc_mala32 300 bash scripts/gpu_pmc.sh r6b_mala32 --sampler mala --no-ess
run pmc_hmc32 300 bash scripts/gpu_pmc.sh r6b_hmc32 --sampler hmc --no-ess
G="SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE;SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_LDS;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_LDS"
export PMC_GROUPS="$G"
run pmc_log128 400 bash scripts/gpu_pmc.sh r6b_log128 --config logistic128 --steps 20 --warmup 2 --no-ess
run pmc_lin512 600 bash scripts/gpu_pmc.sh r6b_lin512 --config linear512 --steps 4 --warmup 100 --no-ess
echo all-done
