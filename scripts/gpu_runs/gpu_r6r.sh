# round 6, call R: config 5 with the second tile's waves at raised priority over the eta MFMAs (prio) against the
# default; phase stamps of the default (DMA spread) build
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6r
mkdir -p $O
AB=$PWD/mcmc.jl_amd/mcmchip/ab
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run lin512 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$AB/libmcmc_hip_prio.so run lin512_prio 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
MCMCHIP_LIB=$AB/libmcmc_hip_stamp.so run stamps512 200 python3 scripts/glm_stamps.py 512 4096 8192
echo all-done
