# round 2 session 4: block-per-chain kernels (2048 < d <= 16384) -- their parity tests, then the full GPU suite.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run s4x_bpc 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -k "block_per_chain" -x -v --timeout 300 --timeout-method thread
run s4x_tests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
echo all-done
