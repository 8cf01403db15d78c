# round 4: config 5 A/B of the eta A-operand lookahead in the 128-wide slices (GLM_ETA_LA 8 / 16 / 32), one box
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4o
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run la8 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
run la16 300 env MCMCHIP_LIB=mcmc.jl_amd/mcmchip/libmcmc_hip_la16.so python3 bench.py --config linear512 --no-cpu-baseline --no-ess
run la32 300 env MCMCHIP_LIB=mcmc.jl_amd/mcmchip/libmcmc_hip_la32.so python3 bench.py --config linear512 --no-cpu-baseline --no-ess
echo all-done
