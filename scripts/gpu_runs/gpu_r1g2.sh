# staged elementwise interleaved with the eta MFMAs; output reserve: GLM parity, config 3/4/5 benches.
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
step g2_tests 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread
step g2_log128 200 python3 bench.py --no-cpu-baseline --config logistic128
step g2_h1024 200 python3 bench.py --no-cpu-baseline --config hmc1024
step g2_lin512 200 python3 bench.py --no-cpu-baseline --config linear512
step g2_lin100 200 python3 bench.py --no-cpu-baseline --config linear512 --d 100 --chains 65536
echo all-done
