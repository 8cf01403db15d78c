# round 6, call C: config-3 A/B of the wave priority in glm_mala1ws's tile loop (s_setprio; variants built with
# -DGLM_WS_PRIO=1: M waves high, =2: V waves high; bitwise-neutral), three alternating runs each
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6c
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
for k in 1 2 3; do
  run base_$k 200 python3 bench.py --config logistic128 --steps 40 --no-cpu-baseline --no-ess
  MCMCHIP_LIB=$PWD/mcmc.jl_amd/mcmchip/ab/libmcmc_hip_prio1.so run prio1_$k 200 python3 bench.py --config logistic128 --steps 40 --no-cpu-baseline --no-ess
  MCMCHIP_LIB=$PWD/mcmc.jl_amd/mcmchip/ab/libmcmc_hip_prio2.so run prio2_$k 200 python3 bench.py --config logistic128 --steps 40 --no-cpu-baseline --no-ess
done
MCMCHIP_LIB=$PWD/mcmc.jl_amd/mcmchip/ab/libmcmc_hip_prio1.so run par1 300 python3 -u -m pytest tests/test_bench_instances.py -m gpu -x -q -k config3 --timeout 120 --timeout-method thread -p no:cacheprovider
MCMCHIP_LIB=$PWD/mcmc.jl_amd/mcmchip/ab/libmcmc_hip_prio2.so run par2 300 python3 -u -m pytest tests/test_bench_instances.py -m gpu -x -q -k config3 --timeout 120 --timeout-method thread -p no:cacheprovider
echo all-done
