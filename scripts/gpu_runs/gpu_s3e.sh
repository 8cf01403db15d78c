# glm_mala1 in its own TU with machine LICM: parity subset + config 3; then the same without scheduling fences
# (mcmchip/variants/libmcmc_hip_f0.so).  Stops at the first failure.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run s3e_tests 300 python3 -u -m pytest tests -m gpu -x -q -k "glm or golden or logistic" --timeout 120 --timeout-method thread
run s3e_log 300 python3 bench.py --no-cpu-baseline --config logistic128
export MCMCHIP_LIB=$PWD/mcmc.jl_amd/mcmchip/variants/libmcmc_hip_f0.so
run s3e_tests_f0 300 python3 -u -m pytest tests -m gpu -x -q -k "glm or golden or logistic" --timeout 120 --timeout-method thread
run s3e_log_f0 300 python3 bench.py --no-cpu-baseline --config logistic128
echo all-done
