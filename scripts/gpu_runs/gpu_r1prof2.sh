# rocprof summaries (trace + FETCH/WRITE passes) of the BASELINE configs after the round-1 kernel work,
# plus RAM benches.
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
bash scripts/gpu_prof.sh r01_logistic128_v2 --config logistic128 || exit $?
bash scripts/gpu_prof.sh r01_hmc1024_v2 --config hmc1024 || exit $?
bash scripts/gpu_prof.sh r01_linear512_v2 --config linear512 || exit $?
bash scripts/gpu_prof.sh r01_d3_v2 --config d3 || exit $?
step p2_ram32 300 python3 bench.py --no-cpu-baseline --config ram32
step p2_ramlin 300 python3 bench.py --no-cpu-baseline --config ramlinear
step p2_readme 300 python3 bench.py --config readme
echo all-done
