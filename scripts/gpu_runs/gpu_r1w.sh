# Round-1 re-entry verification: full GPU suite, smoke, default bench.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
make -C oracle -s
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name exit $rc" | tee -a "$O/steps.txt"
  case $rc in 0|1|2|5) return 0;; *) echo "fatal rc $rc in $name: stopping"; exit $rc;; esac
}
step r1w_tests 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --durations=15
step r1w_smoke 120 python3 -c "import __graft_entry__ as g; g.smoke()"
step r1w_bench 300 python3 bench.py
echo all-done
