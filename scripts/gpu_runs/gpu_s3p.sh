# Session-3 closing check on the committed tree: the whole GPU suite, the smoke and the default bench.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run s3p_tests 800 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run s3p_smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
run s3p_bench 400 python3 bench.py
echo all-done
