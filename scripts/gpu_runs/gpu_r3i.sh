# round 3: scalar kept-step cursor, 52-bit alignbit uniform, angle row from j, uniform-step Philox round 0 --
# suite, benches, rocprof trace + FETCH/WRITE and VALU PMC passes of the metric commands
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3i
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gputests.txt 2>&1 || exit 1
timeout -k 10 240 python bench.py --no-cpu-baseline > $O/bench_metric.json 2> $O/bench_metric.err || exit 1
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_metric20.json 2> $O/bench_metric20.err || exit 1
timeout -k 10 240 python bench.py --config d3 --no-cpu-baseline --no-ess > $O/bench_d3.json 2> $O/bench_d3.err || exit 1
timeout -k 10 240 python bench.py --no-cpu-baseline --no-ess --sampler mala --steps 200 > $O/bench_mala32.json 2> $O/bench_mala32.err || exit 1
timeout -k 10 240 python bench.py --no-cpu-baseline --no-ess --sampler hmc --steps 100 > $O/bench_hmc32.json 2> $O/bench_hmc32.err || exit 1
timeout -k 10 300 python bench.py --config hmc1024 --no-cpu-baseline --no-ess > $O/bench_hmc1024.json 2> $O/bench_hmc1024.err || exit 1
timeout -k 10 600 bash scripts/gpu_prof.sh r3i_metric20 --steps 20 --warmup 5 --no-ess > $O/prof20.log 2>&1 || exit 1
timeout -k 10 600 bash scripts/gpu_pmc.sh r3i_metric20 --steps 20 --warmup 5 --no-ess > $O/pmc20.log 2>&1 || exit 1
timeout -k 10 600 bash scripts/gpu_pmc.sh r3i_metric1000 --no-ess > $O/pmc1000.log 2>&1 || exit 1
echo all-done
