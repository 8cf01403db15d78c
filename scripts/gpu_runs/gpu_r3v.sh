# round 3, session 2: the trajectory-order continuation test, then the roofline profiles of the current step-kernel
# sources (gpu_r3t.sh: VALU PMC of the metric commands / config 2 / config 4, fp64 PMC of configs 3 and 5, trace +
# FETCH/WRITE of the driver's command)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3v
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "trajectory_order or glm" > $O/gputests_glm.txt 2>&1 || exit 1
timeout -k 10 1100 bash scripts/gpu_runs/gpu_r3t.sh > $O/r3t.log 2>&1 || exit 1
echo all-done
