# Session-3 final table: every BASELINE config and the RAM rows on the current build, then a 2-rank gloo
# rehearsal of the multi-rank bench (both ranks on cuda:0).  Stops at the first failure.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run s3j_metric 400 python3 bench.py
run s3j_readme 300 python3 bench.py --config readme
run s3j_d3 300 python3 bench.py --config d3
run s3j_log 300 python3 bench.py --config logistic128
run s3j_h1024 300 python3 bench.py --config hmc1024
run s3j_lin 300 python3 bench.py --config linear512
run s3j_ram32 300 python3 bench.py --no-cpu-baseline --config ram32
run s3j_ramlin 300 python3 bench.py --no-cpu-baseline --config ramlinear
export MCMC_BENCH_BACKEND=gloo
run s3j_tr2 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 200 --warmup 20
echo all-done
