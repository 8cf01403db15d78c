# round 6, call E: glm_mala1ws with unconditional state loads (no masked load + wait per slot) and the regression RAM
# split step at two chains a wave (d <= 256): parity, config-3 and ramlinear128 bench lines, config-3 phase stamps
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6e
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run parity 600 python3 -u -m pytest tests/test_bench_instances.py tests/test_gpu_parity.py tests/test_hook_protocol.py -m gpu -x -q -k "config3 or glm_ram or logistic or mala or ram" --timeout 120 --timeout-method thread -p no:cacheprovider
run log128_a 200 python3 bench.py --config logistic128 --steps 40 --no-cpu-baseline --no-ess
run log128_b 200 python3 bench.py --config logistic128 --steps 40 --no-cpu-baseline --no-ess
run ramlin128 300 python3 bench.py --config ramlinear128 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$PWD/mcmc.jl_amd/mcmchip/ab/libmcmc_hip_wsstamp.so run stamps 200 python3 scripts/ws_stamps.py
echo all-done
