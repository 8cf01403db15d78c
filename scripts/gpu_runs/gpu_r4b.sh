# round 4: 64-wide slices back as the default on the staged-tile image: GLM parity, config 5 / 3 benches, then the
# fp64 + memory PMC passes of config 5
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4b
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run glmtests 600 python3 -u -m pytest tests -m gpu -x -q -k "glm or config3 or config5 or golden or store_leaps or logistic or group" --timeout 300 --timeout-method thread
run lin512 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
G="SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE;SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_LDS;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_LDS;FETCH_SIZE;TCC_HIT_sum TCC_MISS_sum;TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"
PMC_GROUPS="$G" run pmc_lin512 1000 bash scripts/gpu_pmc.sh r4b_lin512 --config linear512 --steps 4 --warmup 100 --no-ess
echo all-done
