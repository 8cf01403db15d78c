# round 4: d-sliced tile loop, LDS-held phase stamps, DMA issued up front (0) vs spread between the eta MFMAs (1)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4f
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
L=mcmc.jl_amd/mcmchip
run st512_0 300 env MCMCHIP_LIB=$L/libmcmc_hip_stamp0.so python3 scripts/glm_stamps.py 512 4096 8192
run st256_0 300 env MCMCHIP_LIB=$L/libmcmc_hip_stamp0.so python3 scripts/glm_stamps.py 256 4096 8192
run lin512_0 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
run lin512_1 300 env MCMCHIP_LIB=$L/libmcmc_hip_spread.so python3 bench.py --config linear512 --no-cpu-baseline --no-ess
echo all-done
