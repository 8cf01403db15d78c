# round 3, session 2: regression models up to d = 1024 (8 slices of 128 coordinates, one X tile buffer) -- GLM parity
# suite, a d = 1024 linear HMCDA bench line, then the fp64 PMC passes of configs 3 and 5 for the new glm.hip hash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3w
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "glm" > $O/gputests_glm.txt 2>&1 || exit 1
timeout -k 10 400 python bench.py --config linear512 --d 1024 --chains 2048 --warmup 30 --steps 10 --no-cpu-baseline --no-ess > $O/bench_linear1024.json 2> $O/bench_linear1024.err || exit 1
G="SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE;SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_LDS;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_SALU"
PMC_GROUPS="$G" timeout -k 10 900 bash scripts/gpu_pmc.sh r3w_log128 --config logistic128 --steps 20 --warmup 2 --no-ess > $O/pmc_log128.log 2>&1 || exit 1
PMC_GROUPS="$G" timeout -k 10 900 bash scripts/gpu_pmc.sh r3w_lin512 --config linear512 --steps 10 --no-ess > $O/pmc_lin512.log 2>&1 || exit 1
echo all-done
