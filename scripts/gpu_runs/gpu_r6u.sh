# round 6, call U: glm_mala1ws' V waves stage the X ring by LDS-DMA (GLM_WS_DMA) against register staging (nodma):
# parity of the single-slice MALA kernels, config 3 twice each, phase stamps
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6u
mkdir -p $O
AB=$PWD/mcmc.jl_amd/mcmchip/ab
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run parity 900 python3 -u -m pytest tests/test_bench_instances.py tests/test_gpu_parity.py tests/test_hook_protocol.py -m gpu -x -q -k "config3 or mala or logistic or glm" --timeout 120 --timeout-method thread -p no:cacheprovider
run log128_a 200 python3 bench.py --config logistic128 --steps 40 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$AB/libmcmc_hip_nodma.so run log128_nodma_a 200 python3 bench.py --config logistic128 --steps 40 --no-cpu-baseline --no-ess
run log128_b 200 python3 bench.py --config logistic128 --steps 40 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$AB/libmcmc_hip_nodma.so run log128_nodma_b 200 python3 bench.py --config logistic128 --steps 40 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$AB/libmcmc_hip_wsstamp.so run stamps 200 python3 scripts/ws_stamps.py
echo all-done
