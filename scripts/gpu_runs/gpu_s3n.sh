# bm_log_u32 on the high word: full parity suite, then the metric bench twice.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run s3n_tests 800 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run s3n_bench 400 python3 bench.py --no-cpu-baseline
run s3n_bench2 400 python3 bench.py --no-cpu-baseline
echo all-done
