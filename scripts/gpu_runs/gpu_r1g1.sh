# single-slice pipelined GLM evaluation (d <= 128): GLM parity tests, config-3 bench, linear d=100/128 bench.
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
step g1_tests 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "glm or logistic or linear or regression"
step g1_log128 300 python3 bench.py --no-cpu-baseline --config logistic128 --steps 40 --warmup 2
step g1_lin512 300 python3 bench.py --no-cpu-baseline --config linear512
echo all-done
