# round 6, call F: config-3 proposal-phase stamps; the RAM split step (d = 128) traced after the eval kernel's
# unconditional state loads
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6f
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
MCMCHIP_LIB=$PWD/mcmc.jl_amd/mcmchip/ab/libmcmc_hip_wsstamp.so run stamps 200 python3 scripts/ws_stamps.py
run ram_parity 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "glm_ram or ram_" --timeout 120 --timeout-method thread -p no:cacheprovider
run prof_ramlinear128 400 bash scripts/gpu_prof.sh r6f_ramlinear128 --config ramlinear128 --no-ess
echo all-done
