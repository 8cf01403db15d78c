# HMC trajectory restructure + FULL wave-per-chain variant + LDS tables for WPC: parity suite and benches.
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
step r1z_tests 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step r1z_h1024 300 python3 bench.py --no-cpu-baseline --config hmc1024
step r1z_hmc 300 python3 bench.py --no-cpu-baseline --sampler hmc
step r1z_mala 300 python3 bench.py --no-cpu-baseline --sampler mala
step r1z_h1024m 300 python3 bench.py --no-cpu-baseline --config hmc1024 --sampler mala --thinning 10
step r1z_h1024r 300 python3 bench.py --no-cpu-baseline --config hmc1024 --sampler rwm --thinning 10
echo all-done
