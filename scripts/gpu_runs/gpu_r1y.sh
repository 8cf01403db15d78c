# guard-free Box-Muller sqrt: GPU parity suite, metric profile (trace + FETCH/WRITE passes), 2-rank gloo rehearsal.
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
step r1y_tests 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step r1y_metric 300 python3 bench.py
bash scripts/gpu_prof.sh r01_metric_v4 || exit $?
MCMC_BENCH_BACKEND=gloo step r1y_tr2 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 200 --warmup 20
echo all-done
