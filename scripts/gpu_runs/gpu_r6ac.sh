# round 6, call AC: the wave RAM update skipping the slots above the pivot row (RAM_WAVE_PRUNE) against computing
# every slot (noprune): RAM parity, ramlinear128, ram256
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6ac
mkdir -p $O
AB=$PWD/mcmc.jl_amd/mcmchip/ab
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run parity 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q -k "ram" --timeout 120 --timeout-method thread -p no:cacheprovider
run ramlin128 200 python3 bench.py --config ramlinear128 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$AB/libmcmc_hip_noprune.so run ramlin128_np 200 python3 bench.py --config ramlinear128 --no-cpu-baseline --no-ess
run ram256 300 python3 bench.py --config ram256 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$AB/libmcmc_hip_noprune.so run ram256_np 300 python3 bench.py --config ram256 --no-cpu-baseline --no-ess
echo all-done
