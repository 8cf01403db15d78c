# round 2 session 5: PMC passes of the kept wave-per-chain RAM kernel (masked columns, prefetch; d=256)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/pmc_r2s5u
mkdir -p $O
A="--no-cpu-baseline --config ram256 --steps 20 --warmup 2 --no-ess"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- python3 bench.py $A > $O/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p2 -o run -- python3 bench.py $A > $O/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/p3 -o run -- python3 bench.py $A > $O/p3.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_WAVES SQ_BUSY_CU_CYCLES SQ_INSTS_SMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/p4 -o run -- python3 bench.py $A > $O/p4.log 2>&1 || exit 1
echo all-done
