cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
MCMC_DEBUG_HOST=1 MCMCHIP_LIB=$PWD/mcmc.jl_amd/mcmchip/libmcmc_hip_dbg.so timeout -k 10 300 python3 scripts/debug_glm1.py > gpurun_out/debug_glm1.log 2>&1 || exit $?
echo skip
echo "rc $?"
