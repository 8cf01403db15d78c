# round 2 session 5: multi-rank rehearsal of the driver's --gpus N path on a 1-GPU box (gloo, both ranks on cuda:0)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
MCMC_BENCH_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/s5t_bench2.log 2>&1 || { tail -30 gpurun_out/s5t_bench2.log; exit 1; }
grep '^{' gpurun_out/s5t_bench2.log | cut -c1-400
echo all-done
