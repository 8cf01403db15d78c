# round 3: occupancy A/B (lpc_rwm d=16 at 3 vs 4 waves/SIMD) + configs 4/5 at their own sizes
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3b
mkdir -p $O
B="python bench.py --d 16 --chains 2097152 --no-cpu-baseline --no-ess --steps 500 --warmup 20"
timeout -k 10 200 $B > $O/d16_w3.json 2> $O/d16_w3.err || exit 1
MCMCHIP_LIB=$PWD/mcmc.jl_amd/mcmchip/libmcmc_hip_w4.so timeout -k 10 200 $B > $O/d16_w4.json 2> $O/d16_w4.err || exit 1
timeout -k 10 200 $B > $O/d16_w3b.json 2> $O/d16_w3b.err || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_configs_full.py > $O/test_configs_full.txt 2>&1 || exit 1
echo all-done
