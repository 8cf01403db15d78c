# round 3: pair-lane kernels -- metric benches first, then the full GPU suite
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 240 python bench.py --no-cpu-baseline > $O/bench_metric.json 2> $O/bench_metric.err || exit 1
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/bench_metric20.json 2> $O/bench_metric20.err || exit 1
timeout -k 10 240 python bench.py --no-cpu-baseline --no-ess --sampler mala --steps 200 > $O/bench_mala32.json 2> $O/bench_mala32.err || exit 1
timeout -k 10 240 python bench.py --no-cpu-baseline --no-ess --sampler hmc --steps 100 > $O/bench_hmc32.json 2> $O/bench_hmc32.err || exit 1
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/gputests.txt 2>&1
echo tests-rc $?

# stall breakdown of the pair metric kernel (driver's command)
PMC_GROUPS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE;SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64" timeout -k 10 400 bash scripts/gpu_pmc.sh r3d_metric20 --steps 20 --warmup 5 --no-ess
echo pmc-rc $?
echo all-done
