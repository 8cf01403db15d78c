# round 3: RAM draws the next rvec into LDS before the fused factor update (the radius tail branches spilled it)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3q
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gputests.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --config ram32 --no-cpu-baseline > $O/bench_ram32.json 2> $O/bench_ram32.err || exit 1
timeout -k 10 300 python bench.py --config ram32 --d 16 --no-cpu-baseline > $O/bench_ram16.json 2> $O/bench_ram16.err || exit 1
timeout -k 10 300 python bench.py --config ram32 --d 8 --no-cpu-baseline > $O/bench_ram8.json 2> $O/bench_ram8.err || exit 1
timeout -k 10 300 python bench.py --config ram256 --no-cpu-baseline > $O/bench_ram256.json 2> $O/bench_ram256.err || exit 1
timeout -k 10 240 python bench.py --no-cpu-baseline --no-ess > $O/bench_metric.json 2> $O/bench_metric.err || exit 1
echo all-done
