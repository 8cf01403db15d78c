# round 2: ESS kernel rewrite (k_ess_tile): bitwise parity tests, then the driver's bench (ESS leg) under a kernel trace.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run r2d_ess 600 python3 -u -m pytest tests -m gpu -k "ess or readme_hmc" -v --timeout 120 --timeout-method thread
run r2d_trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r2d_trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
echo all-done
