# round 6, call O: the d-sliced evaluation's three-phase loop pairing the two tiles' MFMAs with each other's
# elementwise work (GLM_PIPE2) against the three-barrier loop (nopipe): parity, config 5, linear d = 1024 (NW = 8: the
# old loop in both), d = 256
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6o
mkdir -p $O
AB=$PWD/mcmc.jl_amd/mcmchip/ab
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run parity 900 python3 -u -m pytest tests/test_bench_instances.py tests/test_gpu_parity.py -m gpu -x -q -k "config5 or glm or linear or logistic or probit or hmc or mala or rwm" --timeout 120 --timeout-method thread -p no:cacheprovider
run lin512 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$AB/libmcmc_hip_nopipe.so run lin512_nopipe 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
run lin512_b 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$AB/libmcmc_hip_nopipe.so run lin512_nopipe_b 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
echo all-done
