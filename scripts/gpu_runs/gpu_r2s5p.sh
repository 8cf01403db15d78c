# round 2 session 5: full GPU suite, smoke and the driver's bench command on the current build
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/s5p_tests.log 2>&1 || { tail -40 gpurun_out/s5p_tests.log; exit 1; }
tail -2 gpurun_out/s5p_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s5p_smoke.log 2>&1 || { cat gpurun_out/s5p_smoke.log; exit 1; }
tail -1 gpurun_out/s5p_smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s5p_bench.log 2>&1 || { tail gpurun_out/s5p_bench.log; exit 1; }
cut -c1-600 gpurun_out/s5p_bench.log
echo all-done
