# round 4 final check: the whole GPU suite, smoke(), the driver's bench command
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4n
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run tests 1100 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf
run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
echo all-done
