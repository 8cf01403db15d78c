# round 2: double-buffered look-ahead RWM (config 1): its parity tests, then the config-1 bench.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run r2g_tests 600 python3 -u -m pytest tests -m gpu -k "lookahead or readme or golden or single_chain or la_ or bench_instances" -v --timeout 300 --timeout-method thread
run r2g_readme 300 python3 bench.py --config readme
echo all-done
