# round 2, session 4: glm_mala1ws bottleneck split -- config 3 with the V waves' elementwise work removed (e1) and with
# the M waves' MFMAs removed (e2), against the full kernel (results of e1/e2 are wrong by construction: timing only)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run s4g_full 200 python3 bench.py --config logistic128 --no-cpu-baseline --no-ess --steps 50 --warmup 2
MCMCHIP_LIB=$PWD/mcmc.jl_amd/mcmchip/libmcmc_hip_e1.so run s4g_e1 200 python3 bench.py --config logistic128 --no-cpu-baseline --no-ess --steps 50 --warmup 2
MCMCHIP_LIB=$PWD/mcmc.jl_amd/mcmchip/libmcmc_hip_e2.so run s4g_e2 200 python3 bench.py --config logistic128 --no-cpu-baseline --no-ess --steps 50 --warmup 2
echo all-done
