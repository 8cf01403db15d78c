# round 6, call AJ: the tile-pairing parity test over three shapes; config 3 A/B of nontemporal end-of-step state
# stores in glm_mala1ws (GLM_WS_NT=1 build) against the default
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6aj
mkdir -p $O
AB=$PWD/mcmc.jl_amd/mcmchip/ab
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run pairtest 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "tile_pairing" --timeout 120 --timeout-method thread -p no:cacheprovider
MCMCHIP_LIB=$AB/libmcmc_hip_wsnt.so run nt_parity 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_configs_full.py -m gpu -x -q -k "mala or config3 or logistic" --timeout 120 --timeout-method thread -p no:cacheprovider
run log_a 300 python3 bench.py --config logistic128 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$AB/libmcmc_hip_wsnt.so run log_nt 300 python3 bench.py --config logistic128 --no-cpu-baseline --no-ess
run log_a2 300 python3 bench.py --config logistic128 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$AB/libmcmc_hip_wsnt.so run log_nt2 300 python3 bench.py --config logistic128 --no-cpu-baseline --no-ess
echo all-done
