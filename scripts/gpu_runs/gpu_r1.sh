# one GPU session: parity tests, smoke, two bench variants; stop at the first crash/timeout
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name exit $rc" | tee -a "$O/steps.txt"
  case $rc in 0|1|2|5) return 0;; *) echo "fatal rc $rc in $name: stopping"; exit $rc;; esac
}
step r1_pytest_gpu 600 python -m pytest tests -x -q -m gpu
step r1_smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step r1_bench_fused 300 python bench.py --steps 1000 --warmup 50 --no-cpu-baseline
step r1_bench_spl1 300 python bench.py --steps 200 --warmup 10 --spl 1 --no-cpu-baseline
echo all-done
