# round 4: persistent phase-offset RWM pair kernel (MCMCHIP_RWM_PERSIST=1) against the default on the driver's
# metric command, alternating; then parity of the persistent kernel (metric / bench-instance / golden tests)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run d0 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ess
run p0 300 env MCMCHIP_RWM_PERSIST=1 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ess
run d1 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ess
run p1 300 env MCMCHIP_RWM_PERSIST=1 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ess
run p1000 300 env MCMCHIP_RWM_PERSIST=1 python3 bench.py --no-cpu-baseline --no-ess
run d1000 300 python3 bench.py --no-cpu-baseline --no-ess
run ptests 600 env MCMCHIP_RWM_PERSIST=1 python3 -u -m pytest tests -m gpu -x -q -k "metric or bench_instances or golden or readme" --timeout 300 --timeout-method thread
echo all-done
