# round 3: config-2 kernel at 512-thread blocks (2^20 chains = 4 exact rounds of 512 resident blocks, no tail)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3o
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gputests.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --config d3 --no-cpu-baseline --no-ess > $O/bench_d3.json 2> $O/bench_d3.err || exit 1
timeout -k 10 300 python bench.py --config d3 --no-cpu-baseline --no-ess --steps 200 --warmup 20 > $O/bench_d3_200.json 2> $O/bench_d3_200.err || exit 1
echo all-done
