# round 6, call AO: config 5 after the tile skip -- the DMA spread (GLM_DMA_SPREAD 1 / 4 against 2) and the eta
# operand look-ahead (GLM_ETA_LA 4 / 16 against 8), one build each, default first and last
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6ao
mkdir -p $O
AB=$PWD/mcmc.jl_amd/mcmchip/ab
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
B="python3 bench.py --config linear512 --no-cpu-baseline --no-ess"
run def 300 $B
for v in sp1 sp4 la4 la16; do MCMCHIP_LIB=$AB/libmcmc_hip_$v.so run $v 300 $B; done
run def2 300 $B
echo all-done
