# round 6, call Y: the RAM regression update kernel compiled for 4 (default), 5 and 6 waves a SIMD
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6y
mkdir -p $O
AB=$PWD/mcmc.jl_amd/mcmchip/ab
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run parity 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "glm_ram_wave" --timeout 120 --timeout-method thread -p no:cacheprovider
run ramlin128 200 python3 bench.py --config ramlinear128 --no-cpu-baseline --no-ess
for w in 5 6; do MCMCHIP_LIB=$AB/libmcmc_hip_w$w.so run ramlin128_w$w 200 python3 bench.py --config ramlinear128 --no-cpu-baseline --no-ess; done
echo all-done
