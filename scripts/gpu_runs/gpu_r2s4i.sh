# round 2, session 4: exact accept test screened by a single-precision log (gt_det_log) -- full GPU suite, metric bench.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run s4i_tests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run s4i_bench20 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ess
run s4i_bench1000 300 python3 bench.py --steps 1000 --warmup 100 --no-cpu-baseline --no-ess
echo all-done
