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
step r1g_peak 120 scripts/_build/peak_f64
step r1g_log 600 python3 bench.py --config logistic128 --steps 20 --warmup 2 --no-cpu-baseline
step r1g_lin 600 python3 bench.py --config linear512 --steps 4 --warmup 1 --no-cpu-baseline
step r1g_gpu 900 python3 -m pytest tests -q -m gpu -x
echo all-done
