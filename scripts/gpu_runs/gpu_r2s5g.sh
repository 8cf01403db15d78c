# round 2 session 5: RAM update with the next column prefetched
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "ram" > gpurun_out/s5g_tests.log 2>&1 || { tail -30 gpurun_out/s5g_tests.log; exit 1; }
tail -2 gpurun_out/s5g_tests.log
timeout -k 10 200 python3 bench.py --config ram32 --no-ess --no-cpu-baseline > gpurun_out/s5g_ram32.log 2>&1 || exit 1
cut -c1-420 gpurun_out/s5g_ram32.log
timeout -k 10 200 python3 bench.py --config ramlinear --no-ess --no-cpu-baseline > gpurun_out/s5g_ramlin.log 2>&1 || exit 1
cut -c1-300 gpurun_out/s5g_ramlin.log
echo all-done
