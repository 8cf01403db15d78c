# round 5: GPU suite with the regression RAM split step; fp64 PMC + trace of config 3 (det_logi build); the widened
# regression sizes' bench lines
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5c
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run gputests 700 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
G="SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE;SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_LDS;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_LDS"
PMC_GROUPS="$G" run pmc_log128 500 bash scripts/gpu_pmc.sh r5c_log128 --config logistic128 --steps 20 --warmup 2 --no-ess
run trace_log128 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 bench.py --config logistic128 --steps 20 --warmup 2 --no-ess --no-cpu-baseline
run lin1024 500 python3 bench.py --config linear1024 --no-cpu-baseline --no-ess
run ramlin128 300 python3 bench.py --config ramlinear128 --no-cpu-baseline --no-ess
echo all-done
