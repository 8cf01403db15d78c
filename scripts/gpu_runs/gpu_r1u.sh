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
step r1u_ram 300 python3 -m pytest tests/test_gpu_parity.py -q -m gpu -k "test_ram or glm_ram or ess"
step r1u_ram32 300 python3 bench.py --config ram32 --no-cpu-baseline
step r1u_ramlin 300 python3 bench.py --config ramlinear --no-cpu-baseline
step r1u_ramlin20 300 python3 bench.py --config ramlinear --d 20 --no-cpu-baseline
step r1u_ram12 300 python3 bench.py --config ram32 --d 12 --no-cpu-baseline
echo all-done
