# round 3: full bench sweep of the configs on the final metric kernel (cpu_baseline on, bench defaults)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3l
mkdir -p $O
for c in metric readme d3 logistic128 hmc1024 linear512 binomial ram32 ram256 ramlinear; do
  timeout -k 10 400 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || exit 1
  echo "$c done" >> $O/steps.txt
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_metric20.json 2> $O/bench_metric20.err || exit 1
echo all-done
