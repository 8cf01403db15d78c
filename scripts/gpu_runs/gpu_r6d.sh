# round 6, call D: config-3 phase stamps (GLM_WS_STAMP build of glm_mala1ws) and the kernel trace of the RAM split
# step on linear regression d = 128 (ramlinear128)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6d
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
MCMCHIP_LIB=$PWD/mcmc.jl_amd/mcmchip/ab/libmcmc_hip_wsstamp.so run stamps 200 python3 scripts/ws_stamps.py
MCMCHIP_LIB=$PWD/mcmc.jl_amd/mcmchip/ab/libmcmc_hip_wsstamp.so run stamps_small 200 python3 scripts/ws_stamps.py 16384
run prof_ramlinear128 400 bash scripts/gpu_prof.sh r6d_ramlinear128 --config ramlinear128 --no-ess
echo all-done
