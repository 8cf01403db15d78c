# round 2 session 5: wave-per-chain RAM bench (d=256) and the d=32 lane-per-chain RAM bench
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --config ram256 --no-ess > gpurun_out/s5i_ram256.log 2>&1 || { tail gpurun_out/s5i_ram256.log; exit 1; }
cut -c1-2000 gpurun_out/s5i_ram256.log
timeout -k 10 200 python3 bench.py --config ram32 --no-ess > gpurun_out/s5i_ram32.log 2>&1 || exit 1
echo all-done
