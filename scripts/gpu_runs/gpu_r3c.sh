# round 3: pair-lane d<=32 kernels -- VALU probe at 8 waves, occupancy A/B at d=16, full GPU suite, metric benches
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 120 ./scripts/_build/probe_valu_rates > $O/valu_rates.jsonl 2>&1 || exit 1
B="python bench.py --d 16 --chains 2097152 --no-cpu-baseline --no-ess --steps 500 --warmup 20"
timeout -k 10 200 $B > $O/d16_w3.json 2> $O/d16_w3.err || exit 1
MCMCHIP_LIB=$PWD/mcmc.jl_amd/mcmchip/libmcmc_hip_w4.so timeout -k 10 200 $B > $O/d16_w4.json 2> $O/d16_w4.err || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gputests.txt 2>&1 || exit 1
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/bench_metric20.json 2> $O/bench_metric20.err || exit 1
timeout -k 10 240 python bench.py --no-cpu-baseline > $O/bench_metric.json 2> $O/bench_metric.err || exit 1
timeout -k 10 240 python bench.py --no-cpu-baseline --no-ess --sampler mala --steps 200 > $O/bench_mala32.json 2> $O/bench_mala32.err || exit 1
timeout -k 10 240 python bench.py --no-cpu-baseline --no-ess --sampler hmc --steps 100 > $O/bench_hmc32.json 2> $O/bench_hmc32.err || exit 1
echo all-done
