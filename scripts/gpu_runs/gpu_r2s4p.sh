# round 2 session 4: persistent phase-staggered RWM (lpc_rwm_pst) -- bench-instance parity tests, metric benches.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run s4p_tests 600 python3 -u -m pytest tests/test_bench_instances.py -m gpu -x -v --timeout 300 --timeout-method thread
run s4p_b20 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ess
run s4p_b1000 200 python3 bench.py --steps 1000 --warmup 100 --no-cpu-baseline --no-ess
run s4p_b2 200 python3 bench.py --gpus 1 --steps 2 --warmup 5 --no-cpu-baseline --no-ess
echo all-done
