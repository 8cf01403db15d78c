# round 2 session 5: wave-per-chain RAM unconditional column loads (exact wait counts), masked stores: parity + d=256 bench
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "ram" > gpurun_out/s5s_tests.log 2>&1 || { tail -40 gpurun_out/s5s_tests.log; exit 1; }
tail -2 gpurun_out/s5s_tests.log
timeout -k 10 300 python3 bench.py --config ram256 --no-ess > gpurun_out/s5s_ram256.log 2>&1 || { tail gpurun_out/s5s_ram256.log; exit 1; }
cut -c1-2000 gpurun_out/s5s_ram256.log
timeout -k 10 200 python3 bench.py --config ram32 --no-ess > gpurun_out/s5s_ram32.log 2>&1 || exit 1
echo all-done
