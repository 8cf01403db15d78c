# Round-1 results table: every BASELINE config with its CPU baseline; the metric also with --pcie.
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
step tab_metric 400 python3 bench.py --pcie
step tab_readme 300 python3 bench.py --config readme
step tab_d3 300 python3 bench.py --config d3
step tab_log128 300 python3 bench.py --config logistic128
step tab_h1024 300 python3 bench.py --config hmc1024
step tab_lin512 300 python3 bench.py --config linear512
step tab_mala32 300 python3 bench.py --no-cpu-baseline --sampler mala
step tab_hmc32 300 python3 bench.py --no-cpu-baseline --sampler hmc
echo all-done
