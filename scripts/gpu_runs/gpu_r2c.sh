# round 2: mcmc_group (multi-GPU through the C ABI) tests, then the driver's bench command with the VALU roofline.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run r2c_group 600 python3 -u -m pytest tests/test_group.py -m gpu -v --timeout 120 --timeout-method thread
run r2c_bench 400 python3 bench.py --gpus 1 --steps 20 --warmup 5
echo all-done
