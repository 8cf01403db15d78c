# round 3: HMC retry draw no longer CSE'd (VGPR 286 -> 216 at d = 1024); MALA pair-kernel launch variants A/B
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gputests.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --config hmc1024 --no-cpu-baseline --no-ess > $O/bench_hmc1024.json 2> $O/bench_hmc1024.err || exit 1
timeout -k 10 240 python bench.py --no-cpu-baseline --no-ess --sampler hmc --steps 100 > $O/bench_hmc32.json 2> $O/bench_hmc32.err || exit 1
timeout -k 10 240 python bench.py --no-cpu-baseline --no-ess --sampler mala --steps 200 > $O/bench_mala32_m0.json 2> $O/bench_mala32_m0.err || exit 1
for m in 1 2; do
MCMCHIP_LIB=$PWD/mcmc.jl_amd/mcmchip/libmcmc_hip_m$m.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-ess --sampler mala --steps 200 > $O/bench_mala32_m$m.json 2> $O/bench_mala32_m$m.err || exit 1
done
timeout -k 10 240 python bench.py --no-cpu-baseline > $O/bench_metric.json 2> $O/bench_metric.err || exit 1
echo all-done
