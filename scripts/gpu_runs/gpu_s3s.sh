# lookahead RWM with incremental kept-step tracking: small-C tests, whole suite, config 1 bench.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run s3s_small 300 python3 -u -m pytest tests -m gpu -x -q -k "golden or single_chain or seqmc" --timeout 120 --timeout-method thread
run s3s_tests 800 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run s3s_readme 300 python3 bench.py --config readme
run s3s_smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
echo all-done
