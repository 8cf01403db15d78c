# round 6, call Q: the next tile's DMA spread over the eta MFMAs (GLM_DMA_SPREAD stride 2, the new default) against
# stride 1, 3, off (sp0), and stride 2 with eta look-ahead 16: parity of the d-sliced kernels, config 5
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6q
mkdir -p $O
AB=$PWD/mcmc.jl_amd/mcmchip/ab
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run parity 900 python3 -u -m pytest tests/test_bench_instances.py tests/test_gpu_parity.py tests/test_configs_full.py -m gpu -x -q -k "config5 or glm or linear or logistic or probit or hmc" --timeout 120 --timeout-method thread -p no:cacheprovider
run lin512 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
for v in sp0 sp1 sp3 sp2la16; do MCMCHIP_LIB=$AB/libmcmc_hip_$v.so run lin512_$v 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess; done
run lin512_b 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
echo all-done
