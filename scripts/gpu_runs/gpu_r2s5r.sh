# round 2 session 5: A/B experiment, wave RAM pivot with ic = lkk / r (parallel division); bench only
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --config ram256 --no-ess --no-cpu-baseline > gpurun_out/s5r_ram256.log 2>&1 || { tail gpurun_out/s5r_ram256.log; exit 1; }
cut -c1-300 gpurun_out/s5r_ram256.log
echo all-done
