# round 3, session 2: A/B of the metric kernel at 1024-thread blocks (one block and one 56 KB table copy per CU)
# against 512 (two per CU): driver's 20-step command and 1000 steps, alternating libraries; then parity of the
# 1024-thread build on the metric's pair-kernel tests
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3z
mkdir -p $O
L=$PWD/mcmc.jl_amd/mcmchip/libmcmc_hip_t1024.so
for r in 1 2; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ess > $O/b512_20_$r.json 2> $O/b512_20_$r.err || exit 1
  MCMCHIP_LIB=$L timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ess > $O/b1024_20_$r.json 2> $O/b1024_20_$r.err || exit 1
done
timeout -k 10 240 python bench.py --no-cpu-baseline --no-ess > $O/b512_1000.json 2> $O/b512_1000.err || exit 1
MCMCHIP_LIB=$L timeout -k 10 240 python bench.py --no-cpu-baseline --no-ess > $O/b1024_1000.json 2> $O/b1024_1000.err || exit 1
MCMCHIP_LIB=$L timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_bench_instances.py tests/test_golden.py > $O/gputests_t1024.txt 2>&1 || exit 1
echo all-done
