# round 2, session 4: wave-specialised single-slice MALA (glm_mala1ws) -- GLM parity tests, config-3 instance, golden,
# test_syntax.jl cases; config-3 bench; PMC (MFMA/VALU co-execution).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run s4f_tests 400 python3 -u -m pytest tests/test_bench_instances.py tests/test_gpu_parity.py tests/test_golden.py tests/test_reference_syntax.py -m gpu -k "glm or config3 or golden or syntax" -x -q --timeout 120 --timeout-method thread
run s4f_bench 300 python3 bench.py --config logistic128 --no-cpu-baseline --no-ess
run s4f_pmc1 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/s4f_pmc1 -o run -- python3 bench.py --config logistic128 --no-cpu-baseline --no-ess --steps 20 --warmup 2
run s4f_pmc2 200 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $O/s4f_pmc2 -o run -- python3 bench.py --config logistic128 --no-cpu-baseline --no-ess --steps 20 --warmup 2
echo all-done
