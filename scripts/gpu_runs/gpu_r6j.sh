# round 6, call J: 4x4x4_4b regression products with single ds_read_b64 A operands (volatile reads, immediate
# offsets); A/B against the 16x16x4 build (m16) and a deeper operand look-ahead (la12) on configs 3 and 5
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6j
mkdir -p $O
AB=$PWD/mcmc.jl_amd/mcmchip/ab
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run parity 900 python3 -u -m pytest tests/test_bench_instances.py tests/test_gpu_parity.py -m gpu -x -q -k "config3 or config5 or logistic or mala or linear or probit or glm" --timeout 120 --timeout-method thread -p no:cacheprovider
run log128 200 python3 bench.py --config logistic128 --steps 40 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$AB/libmcmc_hip_m16.so run log128_m16 200 python3 bench.py --config logistic128 --steps 40 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$AB/libmcmc_hip_la12.so run log128_la12 200 python3 bench.py --config logistic128 --steps 40 --no-cpu-baseline --no-ess
run lin512 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$AB/libmcmc_hip_m16.so run lin512_m16 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$AB/libmcmc_hip_la12.so run lin512_la12 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
echo all-done
