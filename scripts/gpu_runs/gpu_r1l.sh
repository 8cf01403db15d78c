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
step r1l_gpu 900 python3 -m pytest tests -q -m gpu -x
step r1l_bench 400 python3 bench.py --no-cpu-baseline
step r1l_mala 300 python3 bench.py --no-cpu-baseline --sampler mala --steps 200 --warmup 10
step r1l_hmc 300 python3 bench.py --no-cpu-baseline --sampler hmc --steps 200 --warmup 10
step r1l_d3 300 python3 bench.py --no-cpu-baseline --config d3
echo all-done
