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
step r1t_ess 300 python3 -m pytest tests/test_gpu_parity.py -q -m gpu -k "ess or test_ram or glm_ram"
step r1t_ram32 300 python3 bench.py --config ram32 --cpu-seconds 5
step r1t_ramlin 300 python3 bench.py --config ramlinear --cpu-seconds 5
step r1t_prof 300 rocprofv3 --kernel-trace --stats -d $O/prof_r1t -o run -- python3 bench.py --config ram32 --no-cpu-baseline --steps 50 --warmup 5
echo all-done
