# round 6, call L: glm_mala1ws with and without the M waves' row 3 (nom), config-3 phase stamps; RAM two-stream
# halves parity + bench; the state-rows-past-d regression tests
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6l
mkdir -p $O
AB=$PWD/mcmc.jl_amd/mcmchip/ab
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run parity 900 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "ram or past_d or minus_inf or glm_mala or logistic" --timeout 120 --timeout-method thread -p no:cacheprovider
run log128_a 200 python3 bench.py --config logistic128 --steps 40 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$AB/libmcmc_hip_nom.so run log128_nom_a 200 python3 bench.py --config logistic128 --steps 40 --no-cpu-baseline --no-ess
run log128_b 200 python3 bench.py --config logistic128 --steps 40 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$AB/libmcmc_hip_nom.so run log128_nom_b 200 python3 bench.py --config logistic128 --steps 40 --no-cpu-baseline --no-ess
run ramlin128 200 python3 bench.py --config ramlinear128 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$AB/libmcmc_hip_wsstamp.so run stamps 200 python3 scripts/ws_stamps.py
echo all-done
