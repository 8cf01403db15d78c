# round 3: -2 folded into the Box-Muller radius table, alternating accept draws (pairs) -- suite + metric benches
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gputests.txt 2>&1 || exit 1
timeout -k 10 240 python bench.py --no-cpu-baseline > $O/bench_metric.json 2> $O/bench_metric.err || exit 1
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_metric20.json 2> $O/bench_metric20.err || exit 1
timeout -k 10 240 python bench.py --no-cpu-baseline --no-ess --sampler mala --steps 200 > $O/bench_mala32.json 2> $O/bench_mala32.err || exit 1
timeout -k 10 300 python bench.py --config linear512 --no-cpu-baseline > $O/bench_linear512.json 2> $O/bench_linear512.err || exit 1
timeout -k 10 300 python bench.py --config binomial > $O/bench_binomial.json 2> $O/bench_binomial.err || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_torchrun1.json 2> $O/bench_torchrun1.err || exit 1
MCMC_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_gloo2.json 2> $O/bench_gloo2.err || exit 1
echo all-done
