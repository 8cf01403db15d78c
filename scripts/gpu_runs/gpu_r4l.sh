# round 4: x parked in LDS across the wave RAM update; A/B of two vs three waves per SIMD (MCMCHIP_RAM_WAVES=3) at
# d = 256 and 128, then RAM parity of the default
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4l
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run ram256 300 python3 bench.py --config ram256 --no-cpu-baseline --no-ess
run ram256w3 300 env MCMCHIP_RAM_WAVES=3 python3 bench.py --config ram256 --no-cpu-baseline --no-ess
run ram128 300 python3 bench.py --config ram256 --d 128 --no-cpu-baseline --no-ess
run ram128w3 300 env MCMCHIP_RAM_WAVES=3 python3 bench.py --config ram256 --d 128 --no-cpu-baseline --no-ess
run tests 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q -k "ram_ or _ram" --timeout 300 --timeout-method thread
echo all-done
