# round 4: tile-loop phase stamps of the 128-wide d-slices (config 5 shape, glm_hmc<8, 4>), GLM_STAMP build
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4m
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run st512 300 env MCMCHIP_LIB=mcmc.jl_amd/mcmchip/libmcmc_hip_stamp.so python3 scripts/glm_stamps.py 512 4096 8192
run st512s64 300 env MCMCHIP_GLM_SLICE=64 MCMCHIP_LIB=mcmc.jl_amd/mcmchip/libmcmc_hip_stamp.so python3 scripts/glm_stamps.py 512 4096 8192
echo all-done
