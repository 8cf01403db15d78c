# round 3, session 2 final: bench sweep of every config (bench defaults, cpu_baseline on), in two halves under one
# call's limit: HALF=a or HALF=b
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3y
mkdir -p $O
if [ "$HALF" = "a" ]; then timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gputests.txt 2>&1 || exit 1; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 1; fi
if [ "$HALF" = "a" ]; then CS="metric readme d3 logistic128 hmc1024"; else CS="linear512 binomial ram32 ram256 ramlinear"; fi
for c in $CS; do
  timeout -k 10 400 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || exit 1
  echo "$c done" >> $O/steps.txt
done
if [ "$HALF" = "a" ]; then
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_metric20.json 2> $O/bench_metric20.err || exit 1
fi
echo all-done
