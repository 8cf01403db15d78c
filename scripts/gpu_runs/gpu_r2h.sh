# round 2: few-chain kernels (spec / la) parity, and config-1 kernel time vs the number of kept steps
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -k "lookahead or readme or golden or single_chain or bench_instances or few_chain" -v --timeout 300 --timeout-method thread > $O/r2h_tests.log 2>&1 || exit $?
for th in 1 10 100; do
  timeout -k 10 200 python3 bench.py --config readme --thinning $th --no-cpu-baseline --no-ess > $O/r2h_th$th.log 2>&1 || exit $?
done
echo all-done
