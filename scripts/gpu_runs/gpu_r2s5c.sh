# round 2 session 5: RAM factor row stride an odd multiple of 256 chains (HBM channel spread): ram32 bench
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 bench.py --config ram32 --no-ess --no-cpu-baseline > gpurun_out/s5c_ram32.log 2>&1 || exit 1
cut -c1-420 gpurun_out/s5c_ram32.log
timeout -k 10 200 python3 bench.py --config ramlinear --no-ess --no-cpu-baseline > gpurun_out/s5c_ramlin.log 2>&1 || exit 1
cut -c1-300 gpurun_out/s5c_ramlin.log
echo all-done
