# round 2 session 4: full GPU suite after the config-1 experiments (tree speculation measured and not kept), with
# the screened-accept-test probe and the long / low-acceptance one-chain tests.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run s4u_tests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run s4u_smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
echo all-done
