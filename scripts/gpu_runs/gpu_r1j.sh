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
step r1j_glm 600 python3 -m pytest tests/test_gpu_parity.py -q -x -k "glm or logistic or model_released"
step r1j_log 300 python3 bench.py --config logistic128 --steps 20 --warmup 2 --no-cpu-baseline
step r1j_lin 300 python3 bench.py --config linear512 --steps 4 --warmup 1 --no-cpu-baseline
echo all-done
