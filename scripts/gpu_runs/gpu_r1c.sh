cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name exit $rc" | tee -a "$O/steps.txt"
  case $rc in 0|1|2|5) return 0;; *) echo "fatal rc $rc in $name: stopping"; exit $rc;; esac
}
step r1c_pytest_gpu 900 python3 -m pytest tests -x -q -m gpu
step r1c_bench_hmc1024 300 python3 bench.py --config hmc1024 --steps 100 --warmup 5 --no-cpu-baseline
step r1c_bench_readme 300 python3 bench.py --config readme --steps 1000 --warmup 0 --no-cpu-baseline
step r1c_bench_d3 300 python3 bench.py --config d3 --steps 1000 --warmup 10 --no-cpu-baseline
echo all-done
