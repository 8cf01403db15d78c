# Session-3 re-entry check: parity suite, smoke, default bench, config-3 bench.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name exit $rc" | tee -a "$O/steps.txt"
  case $rc in 0|1|2|5) return 0;; *) echo "fatal rc $rc in $name: stopping"; exit $rc;; esac
}
step s3a_tests 800 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step s3a_smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
step s3a_bench 300 python3 bench.py
step s3a_log 300 python3 bench.py --no-cpu-baseline --config logistic128
echo all-done
