# round 3, session 2: lane / pair HMC kernels take their chains in trajectory-length order too -- full GPU suite,
# smoke, then an A/B of HMCDA on the metric shape (adapted warmup, then timed steps) with the order on and off
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3x
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gputests.txt 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 1
B="python bench.py --sampler hmcda --steps 100 --warmup 100 --no-cpu-baseline --no-ess"
timeout -k 10 300 $B > $O/bench_hmcda32_order.json 2> $O/bench_hmcda32_order.err || exit 1
MCMCHIP_TRAJ_ORDER=0 timeout -k 10 300 $B > $O/bench_hmcda32_noorder.json 2> $O/bench_hmcda32_noorder.err || exit 1
B="python bench.py --sampler hmcda --d 8 --steps 100 --warmup 100 --no-cpu-baseline --no-ess"
timeout -k 10 300 $B > $O/bench_hmcda8_order.json 2> $O/bench_hmcda8_order.err || exit 1
MCMCHIP_TRAJ_ORDER=0 timeout -k 10 300 $B > $O/bench_hmcda8_noorder.json 2> $O/bench_hmcda8_noorder.err || exit 1
echo all-done
