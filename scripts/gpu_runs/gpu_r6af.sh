# round 6, call AF: config 5 with a chain tile that has finished its trajectories skipping its evaluations
# (GLM_TILE_SKIP) and the longest tiles sharing their workgroups with the shortest (tile pairing), against pairing off
# (MCMCHIP_TILE_PAIR=0) and against neither (noskip build, pairing off): parity of the d-sliced HMC / HMCDA kernels
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6af
mkdir -p $O
AB=$PWD/mcmc.jl_amd/mcmchip/ab
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run parity 900 python3 -u -m pytest tests/test_bench_instances.py tests/test_gpu_parity.py tests/test_configs_full.py tests/test_golden.py tests/test_hook_protocol.py -m gpu -x -q -k "config5 or hmc or glm or linear or logistic or probit or golden or leaps or order" --timeout 120 --timeout-method thread -p no:cacheprovider
run lin512 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
MCMCHIP_TILE_PAIR=0 run lin512_nopair 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
MCMCHIP_TILE_PAIR=0 MCMCHIP_LIB=$AB/libmcmc_hip_noskip.so run lin512_old 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
run lin512_b 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
echo all-done
