# IsoDot HMC half kick as (-x) eps (exact path on |x| >= 2^1023): full parity suite, then config 4 and metric-shape HMC.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run s3k_tests 800 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run s3k_h1024 300 python3 bench.py --no-cpu-baseline --config hmc1024
run s3k_hmc32 300 python3 bench.py --no-cpu-baseline --sampler hmc
echo all-done
