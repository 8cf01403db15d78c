# round 6, final validation (after the A/B reverts and rebuild): the whole GPU suite and smoke() on the final tree
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6ap
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run gputests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
echo all-done
