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
step r1h_gpu 900 python3 -m pytest tests -q -m gpu
step r1h_bench 400 python3 bench.py
step r1h_prof_log 900 bash scripts/gpu_prof.sh r01_logistic128 --config logistic128 --steps 20 --warmup 2
step r1h_prof_lin 900 bash scripts/gpu_prof.sh r01_linear512 --config linear512 --steps 4 --warmup 1
echo all-done
