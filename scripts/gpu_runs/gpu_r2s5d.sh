# round 2 session 5: instruction-cache counters of the d=32 RAM step kernel and of the metric RWM kernel
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out/pmc_r2s5d
G="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_IFETCH_LEVEL SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $G --output-format csv -d gpurun_out/pmc_r2s5d/ram -o run -- python3 bench.py --no-cpu-baseline --config ram32 --steps 40 --warmup 4 --no-ess > gpurun_out/pmc_r2s5d/ram.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc $G --output-format csv -d gpurun_out/pmc_r2s5d/rwm -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 2 --no-ess > gpurun_out/pmc_r2s5d/rwm.log 2>&1 || exit 1
echo all-done
