# round 3, session 2: re-check of the tree rebuilt in a fresh container (GPU tests, smoke, the driver's bench
# command), then where the 20-step launch's fixed cost goes (kept rows vs state I/O vs rounds)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3s
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gputests.txt 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 1
for args in "--steps 20 --warmup 5 --thinning 1000" "--steps 40 --warmup 5" "--steps 20 --warmup 5 --chains 524288" "--steps 2 --warmup 5 --thinning 1000" "--steps 100 --warmup 5"; do
  n=$(echo $args | tr -d ' -')
  timeout -k 10 240 python bench.py $args --no-cpu-baseline --no-ess > $O/b_$n.json 2> $O/b_$n.err || exit 1
done
echo all-done
