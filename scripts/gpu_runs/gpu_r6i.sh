# round 6, call I: regression products as v_mfma_f64_4x4x4_4b_f64 (GLM_MFMA4, bitwise the 16x16x4 chains), the
# d-sliced linear model's all-rows weights (GLM_LIN_ALLROWS; _noall: without); the
# unconditional state loads' row-0 fallback; RAM two-stream halves.  Parity, then A/B against the 16x16x4 build
# (mcmchip/ab/libmcmc_hip_m16.so) on configs 3 and 5, RAM on linear regression d = 128
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6i
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run parity 900 python3 -u -m pytest tests/test_bench_instances.py tests/test_gpu_parity.py tests/test_hook_protocol.py tests/test_golden.py -m gpu -x -q -k "config3 or config5 or logistic or mala or linear or probit or glm or ram" --timeout 120 --timeout-method thread -p no:cacheprovider
run log128 200 python3 bench.py --config logistic128 --steps 40 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$PWD/mcmc.jl_amd/mcmchip/ab/libmcmc_hip_m16.so run log128_m16 200 python3 bench.py --config logistic128 --steps 40 --no-cpu-baseline --no-ess
run lin512 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$PWD/mcmc.jl_amd/mcmchip/ab/libmcmc_hip_m16.so run lin512_m16 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$PWD/mcmc.jl_amd/mcmchip/ab/libmcmc_hip_noall.so run lin512_noall 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
run ramlin128 200 python3 bench.py --config ramlinear128 --no-cpu-baseline --no-ess
echo all-done
