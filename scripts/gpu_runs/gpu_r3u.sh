# round 3, session 2: regression HMC/HMCDA chains in trajectory-length order; evaluation counts of RWM/MALA/RAM on the host (no per-wave device-scope atomic on one
# address), one accept-bit atomic per wave in the regression kernels -- suite, then the short-launch benches
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3u
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gputests.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 1
for args in "--steps 2 --warmup 5 --thinning 1000" "--steps 5 --warmup 5" "--steps 40 --warmup 5" "--config binomial" "--config linear512"; do
  n=$(echo $args | tr -d ' -')
  timeout -k 10 240 python bench.py $args --no-cpu-baseline --no-ess > $O/b_$n.json 2> $O/b_$n.err || exit 1
done
echo all-done
