# frexp log_tab + fence knob: parity subset, config 3 with fences (in-tree) and without (variants/libmcmc_hip_f0.so)
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
step s3c_tests 800 python3 -u -m pytest tests -m gpu -x -q -k "detmath or glm or golden or logistic" --timeout 120 --timeout-method thread
step s3c_log_g1 300 python3 bench.py --no-cpu-baseline --config logistic128
export MCMCHIP_LIB=$PWD/mcmc.jl_amd/mcmchip/variants/libmcmc_hip_f0.so
step s3c_log_f0 300 python3 bench.py --no-cpu-baseline --config logistic128
unset MCMCHIP_LIB
step s3c_log_g1b 300 python3 bench.py --no-cpu-baseline --config logistic128
echo all-done
