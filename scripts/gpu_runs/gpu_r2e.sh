# round 2: ESS kernel (unrolled lag loop) parity + timing; the reference's test_syntax.jl configuration on the HIP path.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run r2e_tests 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_reference_syntax.py -m gpu -k "device_ess or syntax" -v --timeout 300 --timeout-method thread
run r2e_trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r2e_trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
echo all-done
