# round 6, call Z: glm_mala1ws draws the next step's proposal normals inside its tile loop (parked in HBM, read by the
# next launch's proposal) against drawing them in the proposal phase (MCMCHIP_GLM_ZN=0): parity, config 3
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6z
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run parity 900 python3 -u -m pytest tests/test_bench_instances.py tests/test_gpu_parity.py tests/test_hook_protocol.py tests/test_task_streams.py tests/test_golden.py -m gpu -x -q -k "config3 or mala or logistic or linear or probit or glm or hook or stream or golden" --timeout 120 --timeout-method thread -p no:cacheprovider
run log128_a 200 python3 bench.py --config logistic128 --steps 40 --no-cpu-baseline --no-ess
MCMCHIP_GLM_ZN=0 run log128_nozn_a 200 python3 bench.py --config logistic128 --steps 40 --no-cpu-baseline --no-ess
run log128_b 200 python3 bench.py --config logistic128 --steps 40 --no-cpu-baseline --no-ess
MCMCHIP_GLM_ZN=0 run log128_nozn_b 200 python3 bench.py --config logistic128 --steps 40 --no-cpu-baseline --no-ess
echo all-done
