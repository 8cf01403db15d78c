# round 3 session 1: VALU issue-cost probe per instruction class + baseline driver-command bench on this box
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 120 ./scripts/_build/probe_valu_rates > $O/valu_rates.jsonl 2>&1 || exit 1
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/bench_metric20.json 2> $O/bench_metric20.err || exit 1
timeout -k 10 240 python bench.py --no-cpu-baseline > $O/bench_metric.json 2> $O/bench_metric.err || exit 1
echo all-done
