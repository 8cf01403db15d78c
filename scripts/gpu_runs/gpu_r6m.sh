# round 6, call M: the wave RAM factor update with two columns' loads in flight (RAM_WAVE_PF = 2) against one (pf1):
# RAM parity, RAM on linear regression d = 128, separable RAM d = 256
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6m
mkdir -p $O
AB=$PWD/mcmc.jl_amd/mcmchip/ab
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run parity 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "ram" --timeout 120 --timeout-method thread -p no:cacheprovider
run ramlin128 200 python3 bench.py --config ramlinear128 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$AB/libmcmc_hip_pf1.so run ramlin128_pf1 200 python3 bench.py --config ramlinear128 --no-cpu-baseline --no-ess
run ram256 300 python3 bench.py --config ram256 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$AB/libmcmc_hip_pf1.so run ram256_pf1 300 python3 bench.py --config ram256 --no-cpu-baseline --no-ess
echo all-done
