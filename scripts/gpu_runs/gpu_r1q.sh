# round-1 evidence refresh: full GPU suite, every bench config, rocprof of the metric kernel
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
step r1q_gpu 900 python3 -m pytest tests -q -m gpu
step r1q_metric 400 python3 bench.py
step r1q_readme 300 python3 bench.py --config readme --no-cpu-baseline
step r1q_d3 300 python3 bench.py --config d3 --no-cpu-baseline
step r1q_log 400 python3 bench.py --config logistic128 --no-cpu-baseline
step r1q_h1024 400 python3 bench.py --config hmc1024 --steps 200 --warmup 10 --no-cpu-baseline
step r1q_lin 400 python3 bench.py --config linear512 --no-cpu-baseline
step r1q_prof 900 bash scripts/gpu_prof.sh r01_metric_v3 --steps 1000 --warmup 100
echo all-done
