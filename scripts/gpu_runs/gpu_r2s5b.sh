# round 2 session 5: RAM parity after the sign fold, ram32 bench, and PMC passes of the d=32 RAM step kernel
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "ram" > gpurun_out/s5b_tests.log 2>&1 || { tail -30 gpurun_out/s5b_tests.log; exit 1; }
tail -2 gpurun_out/s5b_tests.log
timeout -k 10 200 python3 bench.py --config ram32 --no-ess --no-cpu-baseline > gpurun_out/s5b_ram32.log 2>&1 || exit 1
cut -c1-400 gpurun_out/s5b_ram32.log
PMC_GROUPS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE;FETCH_SIZE;WRITE_SIZE;SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_WAVES GRBM_GUI_ACTIVE" bash scripts/gpu_pmc.sh r2s5b_ram --config ram32 --steps 40 --warmup 4 --no-ess || exit $?
echo all-done
