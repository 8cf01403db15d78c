# round 2 session 5: RAM with the next step's S z folded into the factor update (one factor read per step)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "ram" > gpurun_out/s5a_tests.log 2>&1 || { tail -30 gpurun_out/s5a_tests.log; exit 1; }
tail -3 gpurun_out/s5a_tests.log
timeout -k 10 200 python3 bench.py --config ram32 --no-ess > gpurun_out/s5a_ram32.log 2>&1 || exit 1
cat gpurun_out/s5a_ram32.log
timeout -k 10 200 python3 bench.py --config ramlinear --no-ess > gpurun_out/s5a_ramlin.log 2>&1 || exit 1
cat gpurun_out/s5a_ramlin.log
echo all-done
