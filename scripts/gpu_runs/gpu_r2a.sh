# round 2, first call: the whole GPU suite (incl. the new bench-instance and KS tests), smoke, the driver's bench
# command, a rocprofv3 kernel trace of that same command, and the list of PMC counters of this GPU.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
# test failures (rc 1) do not stop the call; a crash, abort or time limit does
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/r2a_tests.log 2>&1
rc=$?; echo "r2a_tests exit $rc"; [ $rc -le 1 ] || exit $rc
run r2a_smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
run r2a_bench 400 python3 bench.py --gpus 1 --steps 20 --warmup 5
run r2a_trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r2a_trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
run r2a_counters 120 rocprofv3 -L
echo all-done
