# round 6, call P: config-5 tile-loop knobs (eta operand look-ahead 16 / 32, the next tile's DMA spread over the eta
# MFMAs) against the default build
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6p
mkdir -p $O
AB=$PWD/mcmc.jl_amd/mcmchip/ab
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run lin512 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
for v in la16 la32 spread; do MCMCHIP_LIB=$AB/libmcmc_hip_$v.so run lin512_$v 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess; done
echo all-done
