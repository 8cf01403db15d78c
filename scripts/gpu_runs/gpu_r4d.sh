# round 4: phase stamps of the d-sliced regression tile loop (GLM_STAMP build), config 5 shape and d = 256
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4d
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run st512 300 env MCMCHIP_LIB=mcmc.jl_amd/mcmchip/libmcmc_hip_stamp.so python3 scripts/glm_stamps.py 512 4096 8192
run st256 300 env MCMCHIP_LIB=mcmc.jl_amd/mcmchip/libmcmc_hip_stamp.so python3 scripts/glm_stamps.py 256 4096 8192
echo all-done
