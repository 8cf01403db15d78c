# round 3, session 2: the final in-tree library (rebuilt after the block-size A/B was reverted) -- GPU suite, smoke and
# the driver's bench command
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3zz
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gputests.txt 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 1
echo all-done
