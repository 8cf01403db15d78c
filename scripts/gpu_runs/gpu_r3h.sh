# round 3: radius polynomials in v (a0..a7 doubles), angle polynomials in j -- suite + benches
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3h
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gputests.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --config hmc1024 --no-cpu-baseline --no-ess > $O/bench_hmc1024.json 2> $O/bench_hmc1024.err || exit 1
timeout -k 10 240 python bench.py --no-cpu-baseline --no-ess --sampler hmc --steps 100 > $O/bench_hmc32.json 2> $O/bench_hmc32.err || exit 1
timeout -k 10 240 python bench.py --no-cpu-baseline --no-ess --sampler mala --steps 200 > $O/bench_mala32.json 2> $O/bench_mala32.err || exit 1
timeout -k 10 240 python bench.py --no-cpu-baseline > $O/bench_metric.json 2> $O/bench_metric.err || exit 1
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_metric20.json 2> $O/bench_metric20.err || exit 1
timeout -k 10 240 python bench.py --config d3 --no-cpu-baseline --no-ess > $O/bench_d3.json 2> $O/bench_d3.err || exit 1
echo all-done
