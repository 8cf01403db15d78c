# round 2 session 4: config 1 on lpc_rwm_tree (256-lane pattern-tree speculation) -- bench-instance + golden parity
# tests, the screened accept test probe, config-1 bench.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run s4r_tests 600 python3 -u -m pytest tests/test_bench_instances.py tests/test_golden.py tests/test_seqmc.py tests/test_gpu_parity.py -m gpu -k "instances or golden or seqmc or tree or lookahead or readme or few_chain or screened" -x -q --timeout 300 --timeout-method thread
run s4r_readme 200 python3 bench.py --config readme
echo all-done
