# round 3: VALU PMC passes (driver's 20-step command, 1000 steps, config 2) on the final metric kernel; gather rate
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3j
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 240 --timeout-method thread -m gpu tests/test_group.py -k gather_rate > $O/gather.txt 2>&1 || exit 1
timeout -k 10 600 bash scripts/gpu_pmc.sh r3j_metric20 --steps 20 --warmup 5 --no-ess > $O/pmc20.log 2>&1 || exit 1
timeout -k 10 600 bash scripts/gpu_pmc.sh r3j_metric1000 --no-ess > $O/pmc1000.log 2>&1 || exit 1
timeout -k 10 600 bash scripts/gpu_pmc.sh r3j_d3 --config d3 --steps 200 --warmup 20 --no-ess > $O/pmcd3.log 2>&1 || exit 1
timeout -k 10 600 bash scripts/gpu_prof.sh r3j_metric1000 --no-ess > $O/prof1000.log 2>&1 || exit 1
echo all-done
