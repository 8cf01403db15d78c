# round 2 session 4 (final metric build: state loads overlapped with table staging): Box-Muller on 512-row radius-log and 1024-row angle tables (+ the screened accept test):
# full GPU suite, metric benches, then the metric kernel's rocprofv3 evidence on the driver's command and at 1000
# steps (kernel trace + FETCH/WRITE passes; VALU PMC passes).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run s4n_tests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run s4n_bench20 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ess
run s4n_bench1000 300 python3 bench.py --steps 1000 --warmup 100 --no-cpu-baseline --no-ess
bash scripts/gpu_prof.sh r2s4n_metric20 --gpus 1 --steps 20 --warmup 5 --no-ess || exit $?
PMC_GROUPS="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE;SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32;SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  bash scripts/gpu_pmc.sh r2s4n_metric20 --gpus 1 --steps 20 --warmup 5 --no-ess || exit $?
bash scripts/gpu_prof.sh r2s4n_metric1000 --no-ess || exit $?
PMC_GROUPS="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE" \
  bash scripts/gpu_pmc.sh r2s4n_metric1000 --no-ess || exit $?
echo all-done
