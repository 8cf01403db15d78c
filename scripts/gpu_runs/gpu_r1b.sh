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
step r1b_bench_full 300 python3 bench.py
for s in mala hmc hmcda; do step r1b_bench_$s 300 python3 bench.py --sampler $s --steps 200 --warmup 10 --no-cpu-baseline; done
step r1b_bench_d3 300 python3 bench.py --d 3 --steps 1000 --warmup 10 --no-cpu-baseline
bash scripts/gpu_prof.sh r1_fused --steps 1000 --warmup 0 || exit $?
bash scripts/gpu_prof.sh r1_spl1 --steps 200 --warmup 0 --spl 1 || exit $?
echo all-done
