# default glm_mala1 without elementwise fences: full parity suite + config 3; variant without the G-product fences
# (mcmchip/variants/libmcmc_hip_gf0.so): parity subset + config 3.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run s3f_tests 800 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run s3f_log 300 python3 bench.py --no-cpu-baseline --config logistic128
export MCMCHIP_LIB=$PWD/mcmc.jl_amd/mcmchip/variants/libmcmc_hip_gf0.so
run s3f_tests_gf0 300 python3 -u -m pytest tests -m gpu -x -q -k "glm or golden or logistic" --timeout 120 --timeout-method thread
run s3f_log_gf0 300 python3 bench.py --no-cpu-baseline --config logistic128
echo all-done
