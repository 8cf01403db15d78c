# round 2, session 4: health check of the restored tree -- full GPU suite, smoke, the driver's bench command.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run s4a_tests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run s4a_smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
run s4a_bench 400 python3 bench.py --gpus 1 --steps 20 --warmup 5
echo all-done
