# round 2 session 5: wave-per-chain RAM continue/shard test
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "ram_wave_continue or ram_limits" > gpurun_out/s5q_tests.log 2>&1 || { tail -40 gpurun_out/s5q_tests.log; exit 1; }
tail -2 gpurun_out/s5q_tests.log
echo all-done
