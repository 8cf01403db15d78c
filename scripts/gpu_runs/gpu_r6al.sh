# round 6, call AL: config 3 with the V waves' late-tile state prefetch (GLM_WS_PF=1, default build) against a
# GLM_WS_PF=0 build, alternating; parity of the default build's single-slice MALA kernels first
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6al
mkdir -p $O
AB=$PWD/mcmc.jl_amd/mcmchip/ab
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run parity 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_configs_full.py tests/test_bench_instances.py -m gpu -x -q -k "mala or config3 or logistic or probit or linear" --timeout 120 --timeout-method thread -p no:cacheprovider
run log_pf 300 python3 bench.py --config logistic128 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$AB/libmcmc_hip_nopf.so run log_nopf 300 python3 bench.py --config logistic128 --no-cpu-baseline --no-ess
run log_pf2 300 python3 bench.py --config logistic128 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$AB/libmcmc_hip_nopf.so run log_nopf2 300 python3 bench.py --config logistic128 --no-cpu-baseline --no-ess
echo all-done
