# round 2 session 6: bench sweep of every config on the rebuilt tree (one line each, cpu_baseline included)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r2s6b
mkdir -p $O
for c in metric d3 readme logistic128 hmc1024 linear512 ram32 ram256 ramlinear; do
  echo "== $c"
  timeout -k 10 240 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || exit 1
done
echo all-done
