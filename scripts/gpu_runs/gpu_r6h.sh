# round 6, call H: glm_mala1ws row 3 of each tile in the M wave (logistic), the -Inf rule per row; glm_ram_wave's
# two-stream halves: parity, config-3 bench, ramlinear128 bench, phase stamps
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6h
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run probe4 120 scripts/_build/probe_mfma4 $O/mfma4_layout.bin
run parity 600 python3 -u -m pytest tests/test_bench_instances.py tests/test_gpu_parity.py tests/test_hook_protocol.py tests/test_golden.py -m gpu -x -q -k "config3 or logistic or mala or linear or probit or glm or ram" --timeout 120 --timeout-method thread -p no:cacheprovider
run log128_a 200 python3 bench.py --config logistic128 --steps 40 --no-cpu-baseline --no-ess
run log128_b 200 python3 bench.py --config logistic128 --steps 40 --no-cpu-baseline --no-ess
run ramlin128 200 python3 bench.py --config ramlinear128 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$PWD/mcmc.jl_amd/mcmchip/ab/libmcmc_hip_wsstamp.so run stamps 200 python3 scripts/ws_stamps.py
echo all-done
