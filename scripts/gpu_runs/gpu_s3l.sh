# the IsoDot overflow-path tests, then the whole GPU suite and the smoke.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run s3l_ovf 300 python3 -u -m pytest tests -m gpu -x -q -k "overflowing" --timeout 120 --timeout-method thread
run s3l_tests 800 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run s3l_smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
echo all-done
